#!/bin/bash
# PMC passes over the weight-gradient microbenchmark (tools/wgrad_bench.py) for one shape filter.
#   bash tools/pmc_wgrad.sh OUT FILTER [lib]
OUT=$1; FLT=$2; LIB=${3:-cosnet_amd/_lib/libcosnet_hip.so}
export WGRAD_CHILD=1 WGRAD_FILTER=$FLT COSNET_HIP_LIB=$LIB
bash tools/pmc_kernel.sh $OUT gemm_kernel -- python3 tools/wgrad_bench.py
