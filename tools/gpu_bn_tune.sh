#!/bin/bash
# BN launch-shape sweep over the whole step (tools/bn_tune_ab.py), one bench run per setting
set -o pipefail
mkdir -p gpurun_out
for spec in default 0=512 0=2048 4=512 4=2048 2=1024 2=4096 6=1024 6=4096 default; do
  echo -n "$spec "
  timeout -k 10 300 python tools/bn_tune_ab.py $spec -- --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],2), round(d['ms_per_step'],2))" || exit 1
done
