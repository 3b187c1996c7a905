#!/bin/bash
# Quick correctness + perf pass for a kernel change (tag = $1): kernel / model GPU tests, the
# default bench line (no CPU baseline), the GEMM breakdown of one eager step.
set -o pipefail
tag=${1:-x}
O=gpurun_out/ab_$tag
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_blocks_bf16.py tests/test_gpu_poisoned_workspace.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?" > $O/rc.txt; exit 1; }
timeout -k 10 400 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?" > $O/rc.txt; exit 1; }
timeout -k 10 300 python tools/gemm_breakdown.py > $O/gemm.txt 2>&1 || { echo "gemm rc=$?" > $O/rc.txt; exit 1; }
echo rc=0 > $O/rc.txt
