#!/bin/bash
# Round-4 GPU pass: changed-area tests, GEMM tile A/B on the layer-3/4 shapes, co-attention
# variant timing, fp8 loss-curve distribution, bench, rocprof trace.
# A test FAILURE (rc 1) does not stop the measurements; any other non-zero status (timeout,
# abort, segfault) ends the script there.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "rc=$rc at $1" > $O/rc.txt; exit $rc; }; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_coatt_fused.py tests/test_gpu_coatt_f8.py tests/test_gpu_poisoned_workspace.py tests/test_gpu_gemm_cfgs.py > $O/tests.log 2>&1; ok tests
timeout -k 10 400 python -u tools/gemm_cold.py l3 19,13,11,21,22,24,25 > $O/gemm_cold_l3.txt 2>&1 || { echo "rc=$? gemm_l3" > $O/rc.txt; exit 1; }
timeout -k 10 300 python -u tools/gemm_cold.py l4_3x3 20,10,23 > $O/gemm_cold_l4.txt 2>&1 || { echo "rc=$? gemm_l4" > $O/rc.txt; exit 1; }
for v in 1 2 3; do for n in 4 5; do
  CN_COATT_VARIANT=$v timeout -k 10 120 python -u tools/coatt_bench.py --n $n >> $O/coatt_v$v.txt 2>&1 || { echo "rc=$? coatt" > $O/rc.txt; exit 1; }
done; done
timeout -k 10 300 python -u tools/fp8_curve_dist.py 5 $O/fp8_curve_dist.json > $O/fp8_curve.log 2>&1 || { echo "rc=$? fp8" > $O/rc.txt; exit 1; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "rc=$? bench" > $O/rc.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 > $O/prof.log 2>&1
echo "rc=$?" > $O/rc.txt
