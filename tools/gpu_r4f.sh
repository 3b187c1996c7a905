#!/bin/bash
# Round-4 GPU pass F: d-split wave-pair co-attention (variant 4) parity + timing + step A/B; SGD
# kernel with all loads in flight (kernel tests + fp32 reference step); the default bench line
# (with the configs[4] fp8 extra).
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_coatt_fused.py tests/test_gpu_kernels.py tests/test_gpu_model.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 4; do
  for n in 4 5; do
    echo -n "variant $v n $n: " >> $O/coatt.txt
    CN_COATT_VARIANT=$v timeout -k 10 120 python tools/coatt_bench.py --n $n 2>/dev/null | tail -1 >> $O/coatt.txt || exit 1
  done
done
timeout -k 10 700 bash tools/ab_env.sh "CN_COATT_VARIANT=1" "CN_COATT_VARIANT=4" > $O/ab.txt 2>&1 || exit 1
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "rc=$? bench" >> $O/rc.txt; exit 1; }
echo "all rc=0" >> $O/rc.txt
