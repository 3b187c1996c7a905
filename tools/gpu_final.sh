#!/bin/bash
# Round-end evidence on one box: rocprofv3 kernel stats of the bench command and the PMC traffic
# passes (both copied into profiles/ on the box so the bench line reads them), then the default
# bench line (with the CPU baseline).  Results under gpurun_out/final/.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 > $O/prof.log 2>&1 || exit 1
cp $(find $O/prof -name "run_kernel_stats.csv" | head -1) $O/kernel_stats.csv || exit 1
bash tools/pmc_run.sh $O/pmc > $O/pmc.log 2>&1 || exit 1
cp $O/kernel_stats.csv profiles/r02_rocprof_kernel_stats_bench_b4_473_final.csv
cp $O/pmc/summary.json profiles/r02_pmc_step_traffic.json
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "rc=$?" > $O/rc.txt
