#!/bin/bash
# partition shards: distributed GPU tests, then bench --shard partitions at N=1 and a 2-rank gloo rehearsal
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_scan.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_dist.log 2>&1 || { tail -60 gpurun_out/t_dist.log; exit 1; }
tail -3 gpurun_out/t_dist.log
timeout -k 10 300 python bench.py --shard partitions --steps 10 --warmup 2 > gpurun_out/bench_ps1.log 2>gpurun_out/bench_ps1.err || { tail -20 gpurun_out/bench_ps1.err; exit 1; }
echo ps1 done
timeout -k 10 400 python bench.py --shard partitions --gpus 2 --backend gloo --steps 10 --warmup 2 > gpurun_out/bench_ps2.log 2>gpurun_out/bench_ps2.err || { tail -20 gpurun_out/bench_ps2.err; exit 1; }
echo ps2 done
