#!/bin/bash
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python bench.py --config bigann100m --data mixture --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline \
  --sweep rescan=0,1 --sweep spill=64,1024 > gpurun_out/bsw.log 2>gpurun_out/bsw.err || { tail -5 gpurun_out/bsw.err; exit 1; }
echo done
