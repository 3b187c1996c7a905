#!/bin/bash
# Split-K slab stores write-through (CN_GEMM_WT=3) vs plain (0): bf16 configs[1] step, three
# alternating rounds
set -o pipefail
mkdir -p gpurun_out/slabwt
for i in 1 2 3; do
  for e in 0 3; do
    CN_GEMM_WT=$e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('bf16 CN_GEMM_WT=$e', round(d['value'],2), 'ms/step %.2f' % d['ms_per_step'])" | tee -a gpurun_out/slabwt/ab.txt || exit 1
  done
done
