#!/bin/bash
# Round-4 GPU pass T: BN launch-shape re-tune on the final tree (cn_bn_set_tuning keys: 0 stats
# blocks, 2 apply blocks, 4 bwd-reduce blocks, 6 bwd-apply blocks), two interleaved rounds.
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for spec in default 2=4096 2=1024 6=4096 6=1024 4=2048 4=512 0=2048 0=512; do
    timeout -k 10 200 python tools/bn_tune_ab.py $spec -- --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', round(d['value'],2), round(d['ms_per_step'],2))" >> $O/ab.txt || exit 1
  done
done
echo "rc=0" > $O/rc.txt
