#!/bin/bash
# k_screen_r diagnosis: phase clocks, same-tile / no-slow-path timing variants, PMC of the base
set -e
mkdir -p gpurun_out
for dat in latent mixture; do
  LIRA_HIP_LIB=variants/rclk.so timeout -k 10 200 python tools/rs_clocks.py sift1m $dat > gpurun_out/rclk_$dat.txt 2>&1
  cat gpurun_out/rclk_$dat.txt | tail -4
done
tools/ab.sh sift1m latent 1 base same noslow
tools/ab.sh sift1m mixture 1 base same noslow
tools/pmc_ab.sh sift1m latent base
python3 -c "import json; j=json.load(open('gpurun_out/pmcab_base/summary.json')); print(json.dumps(j)[:3000])"
