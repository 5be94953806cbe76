#!/bin/bash
# BIGANN-100M latent at HEAD: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (each its own run)
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
PROF_TIMEOUT=900 bash tools/profile_box.sh r04 bigann100m latent mem
echo pmc done
