#!/bin/bash
# Upper bound of an input-halo A loader for the 3x3 gathers (timing only, results wrong):
# tools/gemm_cold.py on the layer-3 / layer-4 3x3 shapes with the product library and with
# var_aonce (CN_PROBE_A_ONCE: A filled for tap 0 only, every other tap reuses it)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for v in cur aonce; do
  L=cosnet_amd/_lib/libcosnet_hip.so; [ $v != cur ] && L=cosnet_amd/_lib/var_$v/libcosnet_hip.so
  echo "== $v" >> $O/aonce.txt
  COSNET_HIP_LIB=$L timeout -k 10 300 python tools/gemm_cold.py 3x3 -1 2>/dev/null >> $O/aonce.txt || exit 1
done
