#!/bin/bash
# spill lists: scan tests, SIFT1M A/B (spill 0 vs default), then BIGANN-100M mixture + latent
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || { tail -40 gpurun_out/t_scan.log; exit 1; }
tail -2 gpurun_out/t_scan.log
for dd in latent mixture; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --data $dd --no-cpu-baseline > gpurun_out/bench_sift_$dd.log 2>gpurun_out/bench_sift_$dd.err || { tail -5 gpurun_out/bench_sift_$dd.err; exit 1; }
done
echo sift done
timeout -k 10 900 python bench.py --config bigann100m --data mixture --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bigann_mixture.log 2>gpurun_out/bench_bigann_mixture.err || { tail -5 gpurun_out/bench_bigann_mixture.err; exit 1; }
echo mixture done
