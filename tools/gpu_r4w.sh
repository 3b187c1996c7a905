#!/bin/bash
# Round-4 GPU pass W: weight-gradient K-split block target (cn_gemm_set_wgrad_target, default 512).
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for spec in default 384 768 1024; do
    timeout -k 10 200 python tools/wgrad_target_ab.py $spec -- --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', round(d['value'],2), round(d['ms_per_step'],2))" >> $O/ab.txt || exit 1
  done
done
echo "rc=0" > $O/rc.txt
