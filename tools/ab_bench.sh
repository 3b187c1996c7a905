#!/bin/bash
# Same-box A/B of the whole train step: current tree vs the tree in abtree/ (git worktree).
for i in 1 2; do
  for t in . abtree; do
    (cd $t && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['value'],2), round(d['ms_per_step'],2))") || exit 1
  done
done
