#!/bin/bash
# q48 arrival counters: zero kernel (CN_Q48_ZERO_KERNEL=1) vs hipMemsetAsync (default): the bench line's
# co-attention fields and step rate, two alternating rounds
set -o pipefail
for i in 1 2; do
  for e in CN_Q48_ZERO_KERNEL=1 CN_Q48_ZERO_KERNEL=0; do
    env $e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline_coattention_train']; c=d['roofline_coattention']
print('$e', round(d['value'],2), 'train frac %.3f fwd %.0f bwd %.0f us/step %.0f | c3 %.1f us' % (r['frac'], r['fwd_tflops'], r['bwd_tflops'], r['us_per_step'], c['us_per_launch']))" || exit 1
  done
done
