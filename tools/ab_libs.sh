#!/bin/bash
# Same-box A/B of the whole train step across built library variants (tools/build_variant.sh):
#   tools/ab_libs.sh variant...   (base = cosnet_amd/_lib/libcosnet_hip.so), two alternating rounds
set -o pipefail
for i in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then L=cosnet_amd/_lib/libcosnet_hip.so; else L=cosnet_amd/_lib/var_$v/libcosnet_hip.so; fi
    COSNET_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],2), round(d['ms_per_step'],2))" || exit 1
  done
done
