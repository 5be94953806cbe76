#!/bin/bash
# One GPU-box session: each step "name|seconds|command" runs under its own
# timeout with its output in gpurun_out/<name>.log; the first failing step ends
# the session (no further GPU work after a fault, abort or time limit).
# usage (through gpurun): bash tools/box_run.sh 'tests|600|python -u -m pytest ...' 'bench|300|python -u bench.py ...'
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -c 2500 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name failed: rc=$rc"; exit $rc; fi
done
