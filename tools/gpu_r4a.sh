#!/bin/bash
# Round-4 first GPU pass: changed-area tests, fp8 loss-curve distribution, bench, rocprof trace.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_coatt_f8.py tests/test_gpu_poisoned_workspace.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/fp8_curve_dist.py 5 $O/fp8_curve_dist.json > $O/fp8_curve.log 2>&1 && \
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 > $O/prof.log 2>&1
echo "rc=$?" > $O/rc.txt
