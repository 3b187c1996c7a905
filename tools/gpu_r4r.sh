#!/bin/bash
# Round-4 GPU pass R: kernel trace of the bench step recorded as split one-stream graphs.
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
export TMPDIR=/tmp
CN_SPLIT_GRAPHS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 --no-roofline > $O/prof.log 2>&1
echo "rc=$?" > $O/rc.txt
