#!/bin/bash
# One parametrised GPU pass (replaces the per-pass gpu_r4*.sh scripts of round 4).
#
#   tools/gpu_pass.sh NAME STEP [STEP ...]
#
# Output goes to gpurun_out/NAME/.  Steps run in order, each under its own time limit, and the
# pass stops at the first failing step (rc in NAME/rc.txt).  A pytest run with failures (rc 1) is
# recorded and the pass goes on (the log names the failure); anything else stops it.
#   tests            the whole GPU suite
#   tests:EXPR       GPU tests selected by -k EXPR
#   file:PATH        GPU tests of one file
#   bench            the default bench line (fp32 / fp8 extras included)
#   bench:ARGS       bench.py ARGS (comma-separated, e.g. bench:--steps,30,--cpu-baseline,0)
#   prof             rocprofv3 kernel trace + stats of the short bench command
#   pmc              the PMC traffic passes of tools/pmc_run.sh
#   smoke            __graft_entry__.smoke()
#   py:SCRIPT[,ARGS] python SCRIPT ARGS (a tools/ probe or A/B script)
#   envbench:VAR=VALUE[,ARGS]  bench.py ARGS with one environment variable set (A/B lines)
#   envprof:VAR=VALUE[,ARGS]   the prof step with one environment variable set (into prof_<i>/)
set -o pipefail
NAME=$1; shift
O=gpurun_out/$NAME
mkdir -p $O
export TMPDIR=/tmp
PY="python -u"
note() { echo "$*" >> $O/rc.txt; }
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  tag=$(printf '%02d_' $i)$(echo "$step" | tr -c 'A-Za-z0-9_.\n-' '_' | cut -c1-60)
  case $kind in
    tests)
      if [ -n "$arg" ]; then sel=(-k "$arg"); else sel=(); fi
      timeout -k 10 900 $PY -m pytest -v --timeout 300 --timeout-method thread -m gpu tests "${sel[@]}" > $O/$tag.log 2>&1
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    file)
      timeout -k 10 600 $PY -m pytest -v --timeout 300 --timeout-method thread -m gpu "$arg" > $O/$tag.log 2>&1
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    bench)
      timeout -k 10 700 $PY bench.py ${arg//,/ } > $O/$tag.json 2> $O/$tag.err
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
        python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 ${arg//,/ } > $O/prof.log 2>&1
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    envprof)
      # envprof:VAR=VALUE[,ARGS]  the prof step with one environment variable set (rocprofv3 takes
      # the program itself after --, so the variable is exported for this step only)
      ev=${arg%%,*}; rest=${arg#*,}; [ "$rest" = "$arg" ] && rest=""
      ( export "$ev"; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$i -o run -- \
        python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 --fp32-extra 0 --fp8-extra 0 ${rest//,/ } > $O/prof_$i.log 2>&1 )
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      timeout -k 10 600 bash tools/pmc_run.sh $O/pmc > $O/pmc.log 2>&1
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 $PY -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    py)
      timeout -k 10 600 $PY ${arg//,/ } > $O/$tag.log 2>&1
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    envbench)
      # envbench:VAR=VALUE,bench-args...  (one environment variable for an A/B bench line)
      ev=${arg%%,*}; rest=${arg#*,}
      env "$ev" timeout -k 10 700 $PY bench.py ${rest//,/ } > $O/$tag.json 2> $O/$tag.err
      rc=$?; note "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    *) note "unknown step $step"; exit 2 ;;
  esac
done
note "done"
