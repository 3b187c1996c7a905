#!/bin/bash
# Write-through output stores (sc1) for the GEMM epilogue (CN_GEMM_WT=1) and the BN apply kernels
# (CN_BN_WT=1) vs plain stores: the bench line's step rate, two alternating rounds; then the
# kernel and bitwise graph-vs-eager tests with both on.
set -o pipefail
mkdir -p gpurun_out/wt
for i in 1 2; do
  for e in "X=0" "CN_GEMM_WT=1" "CN_BN_WT=1" "CN_GEMM_WT=1 CN_BN_WT=1"; do
    env $e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d['roofline_coattention']
print('$e', round(d['value'],2), 'ms/step %.2f gemm ev us %.1f | c3 %.1f us' % (d['ms_per_step'], r['event_avg_launch_us'], c['us_per_launch']))" | tee -a gpurun_out/wt/ab.txt || exit 1
  done
done
CN_GEMM_WT=1 CN_BN_WT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_train_step.py tests/test_gpu_gemm_cfgs.py > gpurun_out/wt/tests.log 2>&1
rc=$?; tail -3 gpurun_out/wt/tests.log; exit $rc
