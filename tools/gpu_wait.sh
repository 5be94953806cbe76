#!/bin/bash
# gpurun, re-submitted ONLY while the pool has no free slot / box (status
# "transient": nothing of the command ran, nothing was charged), every 150 s,
# at most 20 times.  Any run of the command itself -- pass or fail -- ends it.
# usage: tools/gpu_wait.sh <timeout-seconds> <command...>
T=$1; shift
G=/usr/local/graft/bin/gpurun
for attempt in $(seq 1 20); do
  "$G" --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gpu_wait] no free GPU slot (attempt $attempt); retrying in 150 s" >&2
  sleep 150
done
exit 3
