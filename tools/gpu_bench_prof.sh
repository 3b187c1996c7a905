#!/bin/bash
# bench.py default line + rocprofv3 kernel stats of the same bench (tag = $1)
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --cpu-baseline 0 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 8 --warmup 3 --cpu-baseline 0 > gpurun_out/prof_$tag.log 2>&1
echo "rc=$?" > gpurun_out/rc_$tag.txt
