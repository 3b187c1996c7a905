set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 120 python tools/coatt_bench.py > gpurun_out/coatt.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8 -o run -- python bench.py --steps 8 --warmup 3 --cpu-baseline 0 > gpurun_out/prof8.log 2>&1
