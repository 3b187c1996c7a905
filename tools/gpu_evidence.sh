#!/bin/bash
# Round evidence on the current tree (tag = $1): default bench line (with the CPU baseline),
# rocprofv3 kernel stats of the bench, PMC HBM traffic of one eager step.
set -o pipefail
tag=${1:-x}
O=gpurun_out/ev_$tag
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?" > $O/rc.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 > $O/prof.log 2>&1 || { echo "prof rc=$?" > $O/rc.txt; exit 1; }
bash tools/pmc_run.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc rc=$?" > $O/rc.txt; exit 1; }
echo rc=0 > $O/rc.txt
