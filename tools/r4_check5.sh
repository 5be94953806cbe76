#!/bin/bash
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_c5.log 2>&1 || { tail -40 gpurun_out/t_c5.log; exit 1; }
tail -1 gpurun_out/t_c5.log
timeout -k 10 600 python bench.py --config gist1m > gpurun_out/fb_gist.log 2>gpurun_out/fb_gist.err || { tail -5 gpurun_out/fb_gist.err; exit 1; }
echo gist done
timeout -k 10 900 python bench.py --config deep10m --steps 10 > gpurun_out/fb_deep.log 2>gpurun_out/fb_deep.err || { tail -5 gpurun_out/fb_deep.err; exit 1; }
echo deep done
