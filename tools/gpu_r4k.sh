#!/bin/bash
# Round-4 GPU pass K: the tile threshold below which weight-gradient groups split over K
# (CN_WGRAD_GSPLIT: 0 = off, 128 = small layer-1/2 groups, 256 / 512 = also the under-one-round
# groups and the layer-4 1x1 pairs): model tests at the widest setting, same-box step A/B.
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
CN_WGRAD_GSPLIT=4096 timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_model.py tests/test_gpu_train_step.py -k "train_step or model" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_env.sh "CN_WGRAD_GSPLIT=512" "CN_WGRAD_GSPLIT=1024" "CN_WGRAD_GSPLIT=4096" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
