#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pk.log 2>&1 || { tail -40 gpurun_out/t_pk.log; exit 1; }
tail -1 gpurun_out/t_pk.log
for d in mixture latent; do
timeout -k 10 400 python bench.py --data $d --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep seed_pick=0,1,0,1 > gpurun_out/sw_$d.log 2>gpurun_out/sw_$d.err || { tail -5 gpurun_out/sw_$d.err; exit 1; }
timeout -k 10 400 python bench.py --config gist1m --data $d --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep seed_pick=0,1,0,1 > gpurun_out/gsw_$d.log 2>gpurun_out/gsw_$d.err || { tail -5 gpurun_out/gsw_$d.err; exit 1; }
done
timeout -k 10 400 python bench.py --scaling strong --nq 1250 --steps 20 --warmup 3 --no-cpu-baseline --no-exact --no-pipeline --contrast none \
  --sweep seed_pick=0,1,0,1 > gpurun_out/sw_strong.log 2>gpurun_out/sw_strong.err || { tail -5 gpurun_out/sw_strong.err; exit 1; }
echo done
