#!/bin/bash
# Round-4 GPU pass E: SGD kernel with all loads in flight (kernel tests + the fp32 reference step),
# the default bench line (now with the configs[4] fp8 extra), and a kernel-trace of the bench
# command for the SGD / step kernel times.
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "sgd or train_step_fp32_matches_reference" tests/test_gpu_model.py > $O/tests.log 2>&1 || { echo "rc=$? tests" > $O/rc.txt; exit 1; }
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "rc=$? bench" > $O/rc.txt; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 > $O/prof.log 2>&1 || { echo "rc=$? prof" > $O/rc.txt; exit 1; }
echo "rc=0" > $O/rc.txt
