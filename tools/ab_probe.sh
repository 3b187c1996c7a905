#!/bin/bash
# A/B the GEMM variants built by tools/build_variant.sh:
#   bash tools/ab_probe.sh "v1 v2 ..." "shape1 shape2 ..."
for v in $1; do
  for s in $2; do
    COSNET_HIP_LIB=cosnet_amd/_lib/var_$v/libcosnet_hip.so timeout -k 5 60 python3 tools/gemm_probe.py $s -1 100 2>/dev/null | sed "s/^/$v /" || { echo "$v $s FAILED"; exit 1; }
  done
done
