#!/bin/bash
# Selected GPU tests (args: pytest node ids / -k expr), log under gpurun_out/sel_$TAG.log
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -s "$@" > gpurun_out/sel_$TAG.log 2>&1
echo "rc=$?" >> gpurun_out/sel_$TAG.log
