#!/bin/bash
# Round-4 GPU pass V (final evidence of the tree): the full GPU suite, the default bench line (fp32 + fp8 extras), a
# kernel trace + stats of the bench command, smoke.
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "rc=$? bench" > $O/rc.txt; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 > $O/prof.log 2>&1 || { echo "rc=$? prof" > $O/rc.txt; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "rc=$?" > $O/rc.txt
