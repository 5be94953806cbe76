#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c6.log 2>&1 || { tail -40 gpurun_out/t_c6.log; exit 1; }
tail -1 gpurun_out/t_c6.log
timeout -k 10 300 python bench.py --scaling strong --nq 1250 --no-cpu-baseline --contrast none > gpurun_out/fb_strong.log 2>gpurun_out/fb_strong.err || { tail -5 gpurun_out/fb_strong.err; exit 1; }
echo strong done
