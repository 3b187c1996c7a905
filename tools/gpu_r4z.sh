#!/bin/bash
# Round-4 GPU pass Z: ds_read_b64_tr_b8 lane / byte mapping probe (groundwork for fp8 weight
# gradients) and the operand-fill issue-cost probe.
set -o pipefail
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 60 ./tools/probes/tr_b8_probe > $O/tr_b8.txt 2>&1 || { echo "rc=$? tr_b8" > $O/rc.txt; exit 1; }
if [ -x tools/probes/issue_probe ]; then timeout -k 10 120 ./tools/probes/issue_probe > $O/issue.txt 2>&1 || { echo "rc=$? issue" > $O/rc.txt; exit 1; }; fi
echo "rc=0" > $O/rc.txt
