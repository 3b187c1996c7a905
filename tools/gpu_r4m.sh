#!/bin/bash
# Round-4 GPU pass M: one reduce launch per weight-gradient flush (cn_splitk_reduce_multi) --
# kernel tests, model / train-step / block / data-parallel tests, same-box step A/B
# (CN_WGRAD_MULTIRED=0: a reduce launch per problem / group).
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train_step.py tests/test_gpu_blocks_bf16.py \
  tests/test_gpu_dataparallel.py tests/test_gpu_poisoned_workspace.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 bash tools/ab_env.sh "CN_WGRAD_MULTIRED=0" "CN_WGRAD_MULTIRED=1" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
