#!/bin/bash
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c4.log 2>&1 || { tail -40 gpurun_out/t_c4.log; exit 1; }
tail -1 gpurun_out/t_c4.log
rm -f gpurun_out/abo.txt
tools/ab_opts.sh sift1m mixture - spill=0 - spill=0
tools/ab_opts.sh sift1m latent - spill=0
timeout -k 10 900 python bench.py --config bigann100m --data mixture --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bigann_mixture.log 2>gpurun_out/bench_bigann_mixture.err || { tail -5 gpurun_out/bench_bigann_mixture.err; exit 1; }
echo bigmix done
