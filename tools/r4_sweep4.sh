#!/bin/bash
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for d in mixture latent; do
timeout -k 10 400 python bench.py --config gist1m --data $d --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep rounds=4,6,12 --sweep near_rounds=1,3 --sweep xhi=0,1 --sweep qr=128 --sweep near_first=1,4 > gpurun_out/gsw_$d.log 2>gpurun_out/gsw_$d.err || { tail -5 gpurun_out/gsw_$d.err; exit 1; }
done
timeout -k 10 900 python bench.py --config deep10m --steps 5 --warmup 2 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep rounds=4,6,12 --sweep near_rounds=1,3 --sweep xhi=1 > gpurun_out/dsw.log 2>gpurun_out/dsw.err || { tail -5 gpurun_out/dsw.err; exit 1; }
echo done
