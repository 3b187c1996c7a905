#!/bin/bash
# Round 6 A/B: the epilogue prefetch (early EPI 2 pre-BN rows, EPI 3 old-C rows) against the
# previous library (var_base) and against CN_GEMM_PFC=0 (EPI 2 early prefetch kept), two
# alternating rounds of the default bench step (no extras).
set -o pipefail
for i in 1 2; do
  for v in cur base nopfc; do
    L=cosnet_amd/_lib/libcosnet_hip.so; E=""
    [ $v = base ] && L=cosnet_amd/_lib/var_base/libcosnet_hip.so
    [ $v = nopfc ] && E="CN_GEMM_PFC=0"
    env $E COSNET_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --no-roofline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],2), round(d['ms_per_step'],2))" || exit 1
  done
done
