#!/bin/bash
# Round-4 GPU pass B: the full GPU suite, then same-box A/Bs of the whole step (co-attention kernel
# variant, weight-gradient flush point) and the peak-memory probe.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in end layer; do CN_WGRAD_FLUSH=$f timeout -k 10 200 python -u tools/mem_probe.py >> $O/mem.txt 2>&1 || exit 1; done
timeout -k 10 900 bash tools/ab_env.sh "CN_COATT_VARIANT=1" "CN_COATT_VARIANT=2" "CN_COATT_VARIANT=3" "CN_WGRAD_FLUSH=layer" > $O/ab.txt 2>&1
echo "ab rc=$?" >> $O/rc.txt
