#!/bin/bash
# wide re-check: scan tests, then same-box A/B on GIST1M (auto = on) and SIFT1M (auto = off)
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rc.log 2>&1 || { tail -40 gpurun_out/t_rc.log; exit 1; }
tail -2 gpurun_out/t_rc.log
rm -f gpurun_out/abo.txt
tools/ab_opts.sh gist1m latent - recheck=0 - recheck=0
tools/ab_opts.sh gist1m mixture - recheck=0
tools/ab_opts.sh sift1m latent - recheck=1 - recheck=1
tools/ab_opts.sh sift1m mixture - recheck=1
