#!/bin/bash
# Round-3 box run: GPU tests, default bench line, rocprofv3 kernel stats of the bench (tag = $1).
set -o pipefail
tag=${1:-x}
O=gpurun_out/r3_$tag
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?" > $O/rc.txt; exit 1; }
timeout -k 10 400 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?" > $O/rc.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 > $O/prof.log 2>&1 || { echo "prof rc=$?" > $O/rc.txt; exit 1; }
cp $(find $O/prof -name "run_kernel_stats.csv" | head -1) $O/kernel_stats.csv
echo "rc=0" > $O/rc.txt
