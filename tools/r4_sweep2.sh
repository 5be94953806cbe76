#!/bin/bash
# option sweeps at HEAD on one index each (bench.py --sweep): chunking and near-first sizes
set -e
mkdir -p gpurun_out
for d in mixture latent; do
timeout -k 10 400 python bench.py --data $d --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep rounds=3,4,5,6 --sweep near_rounds=1,2,3 --sweep near_first=0,1,2,3,4 > gpurun_out/sw_$d.log 2>gpurun_out/sw_$d.err || { tail -5 gpurun_out/sw_$d.err; exit 1; }
done
timeout -k 10 400 python bench.py --scaling strong --nq 1250 --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep rounds=2,3,4,6,8 --sweep near_rounds=1,2 --sweep near_first=0,1,2,4 > gpurun_out/sw_strong.log 2>gpurun_out/sw_strong.err || { tail -5 gpurun_out/sw_strong.err; exit 1; }
echo done
