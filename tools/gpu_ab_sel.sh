#!/bin/bash
# Selected GPU tests, then a same-box step A/B of the current library against variant libraries.
#   bash tools/gpu_ab_sel.sh TAG "tests/a.py tests/b.py" variant...
set -o pipefail
tag=$1; tests=$2; shift 2
O=gpurun_out/ab_$tag
mkdir -p $O
timeout -k 10 900 python -u -m pytest $tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?" > $O/rc.txt; exit 1; }
bash tools/ab_libs.sh "$@" > $O/ab.txt 2>&1 || { echo "ab rc=$?" > $O/rc.txt; exit 1; }
echo rc=0 > $O/rc.txt
