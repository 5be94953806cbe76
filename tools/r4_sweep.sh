#!/bin/bash
set -e
timeout -k 10 200 python tools/rank_dbg.py 2>&1 | grep -v amdgpu.ids | tail -12
timeout -k 10 500 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_scan.py tests/test_gpu_host_api.py -x -q --timeout 120 --timeout-method thread -m "gpu and not slow" > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
tools/ab.sh gist1m mixture 1 base seed64
tools/ab.sh sift1m mixture 1 base seed64
timeout -k 10 300 python bench.py --config deep10m --steps 3 --warmup 1 --no-cpu-baseline --no-exact --no-pipeline --contrast none > gpurun_out/bench_deep2.log 2>&1
grep -o '"kernels_ms_per_step": {[^}]*}' gpurun_out/bench_deep2.log
