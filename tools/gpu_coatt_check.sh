#!/bin/bash
# co-attention GPU tests + fused-kernel timing at 1, 2, 4, 5 pairs (tools/coatt_bench.py)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/coatt_split.txt
bash tools/gpu_tests_only.sh tests/test_gpu_coatt_fused.py tests/test_gpu_configs.py tests/test_gpu_eval.py tests/test_gpu_kernels.py && \
grep -q "rc=0" gpurun_out/rc.txt && \
for n in 1 2 4 5; do timeout -k 10 120 python tools/coatt_bench.py --n $n 2>/dev/null | tail -1 || exit 1; done > gpurun_out/coatt_split.txt
