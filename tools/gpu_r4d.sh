#!/bin/bash
# Round-4 GPU pass D: in-launch BN finalize (two-level ticket) -- full GPU suite, then a same-box
# step A/B against the separate finalize launches (CN_BN_TICKET=0).
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 700 bash tools/ab_env.sh "CN_BN_TICKET=0" "CN_BN_TICKET=1" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
