#!/bin/bash
# Store-policy A/B on the bf16 configs[1] step, alternating rounds: BN apply outputs plain
# (CN_BN_WT=0) / write-through (1, the default) / non-temporal (3); GEMM C non-temporal
# (CN_GEMM_WT=4) beside the default BN write-through.
set -o pipefail
mkdir -p gpurun_out/stp
R=${1:-3}
for i in $(seq $R); do
  for e in "CN_BN_WT=0" "CN_BN_WT=1" "CN_BN_WT=3" "CN_GEMM_WT=4"; do
    env $e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$e', round(d['value'],2), 'ms/step %.2f' % d['ms_per_step'])" | tee -a gpurun_out/stp/ab.txt || exit 1
  done
done
