#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -2 gpurun_out/t_scan.log
for dat in latent mixture; do
  LIRA_HIP_LIB=variants/rclk.so timeout -k 10 200 python tools/rs_clocks.py sift1m $dat > gpurun_out/rclk_$dat.txt 2>&1
  tail -4 gpurun_out/rclk_$dat.txt
done
tools/ab.sh sift1m latent 2 old base
tools/ab.sh sift1m mixture 2 old base
