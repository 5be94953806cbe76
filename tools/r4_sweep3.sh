#!/bin/bash
set -e
mkdir -p gpurun_out
for d in mixture latent; do
timeout -k 10 400 python bench.py --data $d --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep rounds=3,4,5 --sweep near_rounds=1,2 --sweep near_first=1,2,3,4 --sweep "rounds=3 near_rounds=2" --sweep "rounds=5 near_first=3" > gpurun_out/sw_$d.log 2>gpurun_out/sw_$d.err || { tail -5 gpurun_out/sw_$d.err; exit 1; }
done
echo done
