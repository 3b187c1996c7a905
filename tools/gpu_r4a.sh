#!/bin/bash
# Round-4 first GPU pass: probes (LDS-DMA fill rate, graph-capture stream forks), changed-area
# tests, co-attention variant timing, fp8 loss-curve distribution, bench, rocprof trace.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/probes/fill_rate > $O/fill_rate.txt 2>&1 && \
timeout -k 10 200 python -u tools/probes/capture_fork_probe.py > $O/capture_fork.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_coatt_fused.py tests/test_gpu_coatt_f8.py tests/test_gpu_poisoned_workspace.py > $O/tests.log 2>&1 && \
for v in 1 2 3; do for n in 4 5; do CN_COATT_VARIANT=$v timeout -k 10 120 python -u tools/coatt_bench.py --n $n >> $O/coatt_v$v.txt 2>&1 || exit 1; done; done && \
timeout -k 10 300 python -u tools/fp8_curve_dist.py 5 $O/fp8_curve_dist.json > $O/fp8_curve.log 2>&1 && \
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 > $O/prof.log 2>&1
echo "rc=$?" > $O/rc.txt
