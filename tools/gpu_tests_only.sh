#!/bin/bash
# usage: tools/gpu_tests_only.sh [pytest args...]   (default: the whole -m gpu suite)
set -o pipefail
mkdir -p gpurun_out
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" > gpurun_out/rc.txt
