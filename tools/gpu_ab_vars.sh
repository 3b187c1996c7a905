#!/bin/bash
# Same-box A/B of the default bench step across library builds: cur = the in-tree library, NAME =
# cosnet_amd/_lib/var_NAME/libcosnet_hip.so (a build of another commit / variant).  Two alternating
# rounds.   bash tools/gpu_ab_vars.sh NAME...
set -o pipefail
for i in 1 2; do
  for v in cur "$@"; do
    L=cosnet_amd/_lib/libcosnet_hip.so
    [ $v != cur ] && L=cosnet_amd/_lib/var_$v/libcosnet_hip.so
    COSNET_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],2), round(d['ms_per_step'],2))" || exit 1
  done
done
