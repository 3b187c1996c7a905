#!/bin/bash
# Same-box A/B of the whole train step under environment settings of one tree.
#   bash tools/ab_env.sh "CN_X=0" "CN_X=1 CN_Y=2" ...
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', round(d['value'],2), round(d['ms_per_step'],2))" || exit 1
  done
done
