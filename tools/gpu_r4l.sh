#!/bin/bash
# Round-4 GPU pass L: PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) over one eager step of the
# final tree, for bench.py's roofline.traffic.
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 bash tools/pmc_run.sh $O/pmc > $O/pmc.log 2>&1
echo "rc=$?" > $O/rc.txt
