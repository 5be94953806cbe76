#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_host_api.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -2 gpurun_out/t_scan.log
LIRA_HIP_LIB=variants/rclk.so timeout -k 10 200 python tools/rs_clocks.py sift1m latent > gpurun_out/rclk_latent.txt 2>&1 && tail -5 gpurun_out/rclk_latent.txt
tools/ab.sh sift1m latent 2 prev base
tools/ab.sh sift1m mixture 2 prev base
