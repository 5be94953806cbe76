#!/bin/bash
# round-4 evidence at HEAD: GPU suite, smoke, bench lines (SIFT1M default, strong proxy, GIST1M, DEEP10M, 2-rank gloo)
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/fb_sift.log 2>gpurun_out/fb_sift.err || { tail -5 gpurun_out/fb_sift.err; exit 1; }
echo sift done
timeout -k 10 300 python bench.py --scaling strong --nq 1250 --no-cpu-baseline --contrast none > gpurun_out/fb_strong.log 2>gpurun_out/fb_strong.err || { tail -5 gpurun_out/fb_strong.err; exit 1; }
echo strong done
timeout -k 10 600 python bench.py --config gist1m > gpurun_out/fb_gist.log 2>gpurun_out/fb_gist.err || { tail -5 gpurun_out/fb_gist.err; exit 1; }
echo gist done
timeout -k 10 900 python bench.py --config deep10m --steps 10 > gpurun_out/fb_deep.log 2>gpurun_out/fb_deep.err || { tail -5 gpurun_out/fb_deep.err; exit 1; }
echo deep done
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --no-cpu-baseline --contrast none > gpurun_out/fb_gloo2.log 2>gpurun_out/fb_gloo2.err || { tail -5 gpurun_out/fb_gloo2.err; exit 1; }
echo gloo2 done
