#!/bin/bash
# Round-4 evidence pass: bench line (default flags), rocprofv3 kernel trace + stats of the bench
# command, PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) over one eager step, smoke.
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "rc=$? bench" > $O/rc.txt; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 > $O/prof.log 2>&1 || { echo "rc=$? prof" > $O/rc.txt; exit 1; }
timeout -k 10 800 bash tools/pmc_run.sh $O/pmc > $O/pmc.log 2>&1 || { echo "rc=$? pmc" > $O/rc.txt; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "rc=$?" > $O/rc.txt
