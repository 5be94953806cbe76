#!/bin/bash
# gpurun with ONE delayed re-submit when the box failed while being prepared
# (status "transient": none of the command ran, nothing was charged).  Any
# other outcome -- including failures of the command itself -- is returned as is.
# usage: tools/gpu.sh <timeout-seconds> '<command>'
T=$1; shift
G=/usr/local/graft/bin/gpurun
for attempt in 1 2; do
  "$G" --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] || [ $attempt = 2 ]; then exit $rc; fi
  echo "[gpu.sh] transient box failure; re-submitting once in 60 s" >&2
  sleep 60
done
