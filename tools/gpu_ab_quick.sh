#!/bin/bash
# full -m gpu suite, then a same-box step A/B against the variant libraries named as arguments
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/quick_tests.log 2>&1
echo "tests rc=$?" > gpurun_out/rc_quick.txt
grep -q "tests rc=0" gpurun_out/rc_quick.txt && bash tools/ab_libs.sh "$@" > gpurun_out/ab_quick.txt 2>&1
echo "ab rc=$?" >> gpurun_out/rc_quick.txt
