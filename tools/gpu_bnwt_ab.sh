#!/bin/bash
# BN apply write-through levels: CN_BN_WT=0 (plain stores), 1 (outputs; the default), 2 (also the
# ReLU-mask bytes and the fp8 output copy): bf16 configs[1] step, two alternating rounds, then the
# fp8 B=8 step (configs[4] per GPU) once each
set -o pipefail
mkdir -p gpurun_out/bnwt
for i in 1 2; do
  for e in 0 1 2; do
    CN_BN_WT=$e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('bf16 CN_BN_WT=$e', round(d['value'],2), 'ms/step %.2f' % d['ms_per_step'])" | tee -a gpurun_out/bnwt/ab.txt || exit 1
  done
done
for e in 0 1 2; do
  CN_BN_WT=$e timeout -k 10 400 python bench.py --dtype fp8 --batch 8 --steps 10 --warmup 3 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('fp8 B=8 CN_BN_WT=$e', round(d['value'],2), 'ms/step %.2f' % d['ms_per_step'])" | tee -a gpurun_out/bnwt/ab.txt || exit 1
done
