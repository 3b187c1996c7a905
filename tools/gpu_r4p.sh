#!/bin/bash
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probes/graph_fork_probe.py > $O/probe.txt 2>&1
echo "rc=$?" > $O/rc.txt
