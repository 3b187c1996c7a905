#!/bin/bash
# Round-4 GPU pass F: d-split wave-pair co-attention (variant 4) parity + timing; SGD kernel with
# all loads in flight (kernel tests + the fp32 reference step); same-box step A/B of the
# co-attention variant and of the tile for shallow wide GEMMs (CN_GEMM_SHALLOW).
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_coatt_fused.py tests/test_gpu_kernels.py tests/test_gpu_model.py \
  -k "coatt or fused or flash or pair or sgd or train_step_fp32_matches_reference" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 4; do
  for n in 4 5; do
    echo -n "variant $v n $n: " >> $O/coatt.txt
    CN_COATT_VARIANT=$v timeout -k 10 120 python tools/coatt_bench.py --n $n 2>/dev/null | tail -1 >> $O/coatt.txt || exit 1
  done
done
timeout -k 10 800 bash tools/ab_env.sh "CN_COATT_VARIANT=1" "CN_COATT_VARIANT=4" "CN_GEMM_SHALLOW=11" "CN_GEMM_SHALLOW=1" "CN_GEMM_SHALLOW=9" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
