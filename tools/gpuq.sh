#!/bin/bash
# gpurun, re-submitted (up to 8 times, 75 s apart) ONLY when the pool ran none of
# the command (exit 3: no box / slot free; or status "transient": the box failed
# while being prepared).  Any run of the command itself -- success or failure --
# is returned as is: this never repeats a GPU step that ran.
# usage: tools/gpuq.sh <timeout-seconds> '<command>'   (log: gpurun_out/gpuq.txt)
T=$1; shift
G=/usr/local/graft/bin/gpurun
mkdir -p gpurun_out
for attempt in 1 2 3 4 5 6 7 8; do
  "$G" --timeout "$T" -- "$@" > gpurun_out/gpuq.txt 2>&1
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ $rc -ne 3 ] && [ "$st" != "transient" ] && ! grep -q "no free box\|backing off\|are busy" gpurun_out/gpuq.txt; then
    tail -3 gpurun_out/gpuq.txt; exit $rc
  fi
  echo "[gpuq] attempt $attempt: pool ran nothing (rc=$rc status=$st); retry in 75 s" >&2
  sleep 75
done
tail -3 gpurun_out/gpuq.txt; exit $rc
