#!/bin/bash
# Same-box A/B of environment settings on a chosen bench line, two alternating rounds:
#   bash tools/ab_env_args.sh "BENCH ARGS" "CN_X=0" "CN_X=1" ...
set -o pipefail
ARGS=$1; shift
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py $ARGS --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', round(d['value'],2), round(d['ms_per_step'],2))" || exit 1
  done
done
