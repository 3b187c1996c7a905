#!/bin/bash
# Round-4 GPU pass Q: the step recorded as one-stream graphs per phase and stream (CN_SPLIT_GRAPHS)
# -- bitwise graph-vs-eager tests, host-side replay probe, same-box step A/B.
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_train_step.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CN_SPLIT_GRAPHS=1 PROBE_TOY=0 timeout -k 10 200 python -u tools/probes/graph_relaunch_probe.py > $O/probe.txt 2>&1 || exit 1
timeout -k 10 800 bash tools/ab_env.sh "CN_SPLIT_GRAPHS=0" "CN_SPLIT_GRAPHS=1" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
