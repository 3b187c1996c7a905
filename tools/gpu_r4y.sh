#!/bin/bash
# Round-4 GPU pass Y: GEMM grouped tile order (CN_GEMM_GROUP_M 4 / 8 (base) / 16), whole step.
set -o pipefail
O=gpurun_out/r4y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 bash tools/ab_libs.sh gm4 gm16 > $O/ab.txt 2>&1
echo "rc=$?" > $O/rc.txt
