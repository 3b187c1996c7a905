#!/bin/bash
# Round-4 GPU pass X: BN minimum rows per thread (cn_bn_set_tuning keys 1 stats, 3 apply, 5 bwd
# reduce, 7 bwd apply) on the final tree.
set -o pipefail
O=gpurun_out/r4x
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for spec in default 3=8 7=8 5=8 1=16 3=8,7=8; do
    timeout -k 10 200 python tools/bn_tune_ab.py $spec -- --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', round(d['value'],2), round(d['ms_per_step'],2))" >> $O/ab.txt || exit 1
  done
done
echo "rc=0" > $O/rc.txt
