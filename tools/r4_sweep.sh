#!/bin/bash
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_host_api.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
for dat in latent mixture; do
tools/ab_opts.sh sift1m $dat "-" "rounds=4 near_rounds=1" "rounds=4 near_rounds=2"
done
BENCH_ARGS="--nq 1250" tools/ab_opts.sh sift1m mixture "-" "rounds=8" "rounds=8 near_rounds=2"
