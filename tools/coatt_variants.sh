#!/bin/bash
# Time the fused co-attention kernel for each built variant library (tools/build_variant.sh).
# usage: tools/coatt_variants.sh [--n PAIRS] variant...
set -o pipefail
N=4
if [ "$1" = "--n" ]; then N=$2; shift 2; fi
for v in base "$@"; do
  if [ $v = base ]; then L=cosnet_amd/_lib/libcosnet_hip.so; else L=cosnet_amd/_lib/var_$v/libcosnet_hip.so; fi
  echo -n "$v "
  COSNET_HIP_LIB=$L timeout -k 10 120 python tools/coatt_bench.py --n $N 2>/dev/null | tail -1 || exit 1
done
