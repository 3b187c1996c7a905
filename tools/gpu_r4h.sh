#!/bin/bash
# Round-4 GPU pass H: grouped weight gradients split over K for the small (layer-1/2) shapes --
# kernel tests, model-level tests, same-box step A/B (CN_WGRAD_GSPLIT=0 issues them one by one).
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train_step.py tests/test_gpu_blocks_bf16.py \
  -k "wgrad or train_step or model or bottleneck or block" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 bash tools/ab_env.sh "CN_WGRAD_GSPLIT=0" "CN_WGRAD_GSPLIT=1" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
