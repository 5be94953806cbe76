#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py --config gist1m --steps 10 --warmup 2 > gpurun_out/bench_gist.log 2>gpurun_out/bench_gist.err || { tail -5 gpurun_out/bench_gist.err; exit 1; }
echo gist done
