#!/bin/bash
# replay-after-eager check, then the partition-shard bench (N=1, then 2 gloo ranks)
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/replay_repro.py mixture > gpurun_out/repro.log 2>&1 || { tail -30 gpurun_out/repro.log; exit 1; }
cat gpurun_out/repro.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --shard partitions --steps 10 --warmup 2 > gpurun_out/bench_ps1.log 2>gpurun_out/bench_ps1.err || { tail -20 gpurun_out/bench_ps1.err; exit 1; }
echo ps1 done
timeout -k 10 400 python bench.py --shard partitions --gpus 2 --backend gloo --steps 10 --warmup 2 > gpurun_out/bench_ps2.log 2>gpurun_out/bench_ps2.err || { tail -20 gpurun_out/bench_ps2.err; exit 1; }
echo ps2 done
