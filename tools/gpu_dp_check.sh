#!/bin/bash
# DP GPU tests + a 2-rank gloo rehearsal of bench.py on the box's one GPU + the default bench line
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/rc_dpc.txt
bash tools/gpu_tests_only.sh tests/test_gpu_dataparallel.py && grep -q "rc=0" gpurun_out/rc.txt && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo --cpu-baseline 0 \
  > gpurun_out/bench_dp2_gloo.json 2> gpurun_out/bench_dp2_gloo.err && \
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
echo "rc=$?" > gpurun_out/rc_dpc.txt
