#!/bin/bash
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_host_api.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
LIRA_HIP_LIB=variants/rclk.so timeout -k 10 200 python tools/rs_clocks.py sift1m latent > gpurun_out/rclk_latent.txt 2>&1 && tail -3 gpurun_out/rclk_latent.txt
for dat in latent mixture; do
tools/ab_opts.sh sift1m $dat "near_first=0" "-" "near_first=1" "near_first=4"
done
BENCH_ARGS="--nq 1250" tools/ab_opts.sh sift1m mixture "near_first=0" "-" "near_first=1" "near_first=4"
