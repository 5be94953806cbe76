#!/bin/bash
# checkpoint: every GPU test (full-size included), smoke, then rocprof evidence for SIFT1M
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
PROF_TIMEOUT=200 timeout -k 10 900 tools/profile_all.sh r04 sift1m:latent sift1m:mixture
