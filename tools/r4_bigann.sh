#!/bin/bash
# BIGANN-100M (n_mul = 2, 207 GB index) bench lines at HEAD + the latent PMC memory passes
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python bench.py --config bigann100m --data latent --steps 5 --warmup 2 > gpurun_out/bench_bigann_latent.log 2>gpurun_out/bench_bigann_latent.err || { tail -5 gpurun_out/bench_bigann_latent.err; exit 1; }
echo latent done
timeout -k 10 900 python bench.py --config bigann100m --data mixture --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bigann_mixture.log 2>gpurun_out/bench_bigann_mixture.err || { tail -5 gpurun_out/bench_bigann_mixture.err; exit 1; }
echo mixture done
