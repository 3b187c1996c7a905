#!/bin/bash
# Round-4 GPU pass B: the full GPU suite, GEMM tile A/B (layer-3 N = 256 products, isolated and in
# the step), weight-gradient flush A/B and the peak-memory probe.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_cold.py l3 19,11,24,25 > $O/gemm_cold_l3.txt 2>&1 || exit 1
for f in end layer; do CN_WGRAD_FLUSH=$f timeout -k 10 200 python -u tools/mem_probe.py >> $O/mem.txt 2>&1 || exit 1; done
timeout -k 10 1100 bash tools/ab_env.sh "CN_GEMM_N256=19" "CN_GEMM_N256=11" "CN_GEMM_N256=24" "CN_GEMM_N256=25" "CN_WGRAD_FLUSH=layer" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
