#!/bin/bash
# Submit one gpurun command, re-submitting ONLY while the pool reports no free box / slot (status
# "transient": nothing ran, nothing charged).  Any call that actually ran -- pass or fail -- ends
# the loop; its output is left in gpurun_out/ as usual.
#   tools/gpurun_when_free.sh <timeout_s> <command> [max_tries]
T=$1; CMD=$2; N=${3:-12}
for i in $(seq 1 $N); do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout $T -- "$CMD"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[when_free] no box (try $i), waiting" >&2
  sleep 150
done
exit 3
