#!/bin/bash
# Same-box A/B of an environment switch on the default bench line (no CPU baseline):
#   bash tools/gpu_env_ab.sh TAG "ENV_A" "ENV_B" [reps]   e.g. "CN_GEMM_HEUR=1" "CN_GEMM_HEUR=0"
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}
O=gpurun_out/envab_$TAG
mkdir -p $O
: > $O/summary.txt
for i in $(seq 1 $R); do
  for side in A B; do
    if [ $side = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/$side$i.json 2> $O/$side$i.err || { echo "bench $side$i failed" >> $O/summary.txt; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/$side$i.json').read().strip().splitlines()[-1]); print('$side', '$E', d['value'], d['ms_per_step'])" >> $O/summary.txt
  done
done
cat $O/summary.txt
