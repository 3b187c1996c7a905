#!/bin/bash
# Round-4 GPU pass N: graph re-launch probe (does a replay wait for the previous one?).
set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probes/graph_relaunch_probe.py > $O/probe.txt 2>&1
echo "rc=$?" > $O/rc.txt
