#!/bin/bash
# Round-2 GPU pass: full -m gpu suite, default bench line, per-shape GEMM breakdown.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" > gpurun_out/rc.txt
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python tools/gemm_breakdown.py > gpurun_out/gemm_breakdown.txt 2>&1
echo "bench rc=$?" >> gpurun_out/rc.txt
