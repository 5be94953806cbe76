#!/bin/bash
# bench lines for the non-headline configs at HEAD (profiles/r04_bench_*.json)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --config gist1m --steps 10 --warmup 2 > gpurun_out/bench_gist.log 2>gpurun_out/bench_gist.err || { tail -5 gpurun_out/bench_gist.err; exit 1; }
echo gist done
timeout -k 10 600 python bench.py --config deep10m --steps 5 --warmup 2 > gpurun_out/bench_deep.log 2>gpurun_out/bench_deep.err || { tail -5 gpurun_out/bench_deep.err; exit 1; }
echo deep done
timeout -k 10 300 python bench.py --scaling strong --nq 1250 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_strong.log 2>gpurun_out/bench_strong.err || { tail -5 gpurun_out/bench_strong.err; exit 1; }
echo strong done
