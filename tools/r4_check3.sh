#!/bin/bash
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c3.log 2>&1 || { tail -40 gpurun_out/t_c3.log; exit 1; }
tail -1 gpurun_out/t_c3.log
timeout -k 10 600 python bench.py > gpurun_out/fb_sift.log 2>gpurun_out/fb_sift.err || { tail -5 gpurun_out/fb_sift.err; exit 1; }
echo sift done
timeout -k 10 900 python bench.py --config bigann100m --data mixture --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bigann_mixture.log 2>gpurun_out/bench_bigann_mixture.err || { tail -5 gpurun_out/bench_bigann_mixture.err; exit 1; }
echo bigmix done
timeout -k 10 900 python bench.py --config bigann100m --data latent --steps 5 --warmup 2 > gpurun_out/bench_bigann_latent.log 2>gpurun_out/bench_bigann_latent.err || { tail -5 gpurun_out/bench_bigann_latent.err; exit 1; }
echo biglat done
