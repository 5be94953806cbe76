#!/bin/bash
set -e
mkdir -p gpurun_out
for dat in latent mixture; do
  LIRA_HIP_LIB=variants/rclk.so timeout -k 10 200 python tools/rs_clocks.py sift1m $dat > gpurun_out/rclk_$dat.txt 2>&1 || { tail -20 gpurun_out/rclk_$dat.txt; exit 1; }
  tail -5 gpurun_out/rclk_$dat.txt
done
