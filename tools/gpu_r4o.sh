#!/bin/bash
# Round-4 GPU pass O: graph re-launch behaviour of the real step with 1 / 2 alternating recordings
# and with the encoders on one stream; same-box step A/B of the same settings.
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
for cfg in "PROBE_BUFFERS=1" "PROBE_BUFFERS=2" "PROBE_BUFFERS=1 CN_CONCURRENT_ENCODERS=0" "PROBE_BUFFERS=2 CN_CONCURRENT_ENCODERS=0"; do
  echo "== $cfg" >> $O/probe.txt
  env PROBE_TOY=0 $cfg timeout -k 10 200 python -u tools/probes/graph_relaunch_probe.py 2>&1 | grep -v amdgpu.ids >> $O/probe.txt || exit 1
done
timeout -k 10 900 bash tools/ab_env.sh "CN_GRAPH_BUFFERS=1" "CN_GRAPH_BUFFERS=2" "CN_GRAPH_BUFFERS=1 CN_CONCURRENT_ENCODERS=0" "CN_GRAPH_BUFFERS=2 CN_CONCURRENT_ENCODERS=0" > $O/ab.txt 2>&1
echo "rc=$?" > $O/rc.txt
