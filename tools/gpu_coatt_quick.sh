#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_coatt_fused.py > gpurun_out/coatt_tests.log 2>&1 || { echo "tests failed" > gpurun_out/rc3.txt; exit 1; }
bash tools/coatt_variants.sh --n 4 qreg kpf4 > gpurun_out/cvar4.txt 2>&1 && bash tools/coatt_variants.sh --n 5 qreg > gpurun_out/cvar5.txt 2>&1 && \
bash tools/ab_libs.sh zr0 > gpurun_out/ab_zr.txt 2>&1
echo "rc=$?" > gpurun_out/rc3.txt
