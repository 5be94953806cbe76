#!/bin/bash
# final round-4 evidence at HEAD: SIFT1M PMC re-profile, GPU suite, smoke, default bench line (with the fresh records)
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/profile_box.sh r04 sift1m latent all > /dev/null
bash tools/profile_box.sh r04 sift1m mixture all > /dev/null
echo profiled
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
