#!/bin/bash
# bench.py over dtype x batch (no CPU baseline): bf16/fp8 at B=4 (configs[1]) and B=8 (configs[4]'s per-GPU batch)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_matrix.txt
for dt in bf16 fp8; do for b in 4 8; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline --dtype $dt --batch $b > gpurun_out/bm_${dt}_${b}.json 2> gpurun_out/bm_${dt}_${b}.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bm_${dt}_${b}.json').read().strip().splitlines()[-1]); print('$dt B=$b', round(d['value'],1), 'pairs/s', round(d['ms_per_step'],2), 'ms/step')" >> gpurun_out/bench_matrix.txt
done; done
