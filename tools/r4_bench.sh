#!/bin/bash
# the driver's default bench line + the 2-rank rehearsal (gloo, both ranks on the box's one GPU)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
tail -c 400 gpurun_out/bench_default.log
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_g2.log 2>gpurun_out/bench_g2.err || { tail -20 gpurun_out/bench_g2.err; exit 1; }
tail -c 300 gpurun_out/bench_g2.log
