#!/bin/bash
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python bench.py --config deep10m --steps 5 --warmup 2 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep two_phase=0,2 --sweep share=0 --sweep qr=32 --sweep split=0 --sweep prune=0 --sweep rounds=2,16 --sweep seed=0 > gpurun_out/dsw.log 2>gpurun_out/dsw.err || { tail -5 gpurun_out/dsw.err; exit 1; }
echo done
