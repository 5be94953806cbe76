#!/bin/bash
# after the fill-kernel fix: scan + distributed GPU tests, partition-shard bench N=1 and 2 gloo ranks
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_distributed.py tests/test_gpu_host_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_fix.log 2>&1 || { tail -40 gpurun_out/t_fix.log; exit 1; }
tail -2 gpurun_out/t_fix.log
timeout -k 10 300 python bench.py --shard partitions --steps 10 --warmup 2 > gpurun_out/bench_ps1.log 2>gpurun_out/bench_ps1.err || { tail -20 gpurun_out/bench_ps1.err; exit 1; }
echo ps1 done
timeout -k 10 400 python bench.py --shard partitions --gpus 2 --backend gloo --steps 10 --warmup 2 > gpurun_out/bench_ps2.log 2>gpurun_out/bench_ps2.err || { tail -20 gpurun_out/bench_ps2.err; exit 1; }
echo ps2 done
