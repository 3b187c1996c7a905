#!/bin/bash
# BN apply store policy A/B: CN_BN_WT=0 (plain stores), 1 (write-through outputs; the default),
# 2 (also the ReLU-mask bytes and the fp8 output copy), 3 (non-temporal stores).
#   tools/gpu_bnwt_ab.sh "0 1 3" [rounds]      bf16 configs[1] step, alternating rounds
set -o pipefail
mkdir -p gpurun_out/bnwt
LV=${1:-"0 1 2"}; R=${2:-2}
for i in $(seq $R); do
  for e in $LV; do
    CN_BN_WT=$e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('bf16 CN_BN_WT=$e', round(d['value'],2), 'ms/step %.2f' % d['ms_per_step'])" | tee -a gpurun_out/bnwt/ab2.txt || exit 1
  done
done
