#!/bin/bash
# round-4 first GPU check: scan parity (k_screen_r default) + rscreen A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/t_scan.log 2>&1
rc=$?
tail -15 gpurun_out/t_scan.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
tools/ab_opts.sh sift1m mixture "rscreen=0" "rscreen=1" && tools/ab_opts.sh sift1m latent "rscreen=0" "rscreen=1"
