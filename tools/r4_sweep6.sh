#!/bin/bash
set -e
mkdir -p gpurun_out
for d in mixture latent; do
timeout -k 10 400 python bench.py --data $d --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep seed_tiles=4,2,4,2 > gpurun_out/sw_$d.log 2>gpurun_out/sw_$d.err || { tail -5 gpurun_out/sw_$d.err; exit 1; }
done
timeout -k 10 400 python bench.py --scaling strong --nq 1250 --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep seed_tiles=4,2,4,2 > gpurun_out/sw_strong.log 2>gpurun_out/sw_strong.err || { tail -5 gpurun_out/sw_strong.err; exit 1; }
echo done
