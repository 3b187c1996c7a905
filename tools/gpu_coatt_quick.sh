#!/bin/bash
# co-attention tests, fused-kernel timing for base and variant libraries, whole-step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_coatt_fused.py tests/test_gpu_configs.py > gpurun_out/coatt_tests.log 2>&1 || { echo "tests failed" > gpurun_out/rc3.txt; exit 1; }
bash tools/coatt_variants.sh --n 5 "$@" > gpurun_out/cvar5.txt 2>&1 && bash tools/coatt_variants.sh --n 4 "$@" > gpurun_out/cvar4.txt 2>&1 && \
bash tools/ab_libs.sh "$@" > gpurun_out/ab_quick.txt 2>&1
echo "rc=$?" > gpurun_out/rc3.txt
