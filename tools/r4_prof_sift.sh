#!/bin/bash
# rocprofv3 trace + PMC passes for SIFT1M both distributions at HEAD, then the default bench line with the fresh records
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
bash tools/profile_box.sh r04 sift1m latent all > /dev/null
echo latent profiled
bash tools/profile_box.sh r04 sift1m mixture all > /dev/null
echo mixture profiled
