#!/bin/bash
# Round-4 GPU pass U: BN backward-reduce block count below the pass-T optimum (512), and combined.
set -o pipefail
O=gpurun_out/r4u
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for spec in default 4=512 4=384 4=256 4=512,0=512 4=512,6=1024; do
    timeout -k 10 200 python tools/bn_tune_ab.py $spec -- --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', round(d['value'],2), round(d['ms_per_step'],2))" >> $O/ab.txt || exit 1
  done
done
echo "rc=0" > $O/rc.txt
