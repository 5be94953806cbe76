#!/bin/bash
set -e
rm -f gpurun_out/ab.txt
tools/ab.sh sift1m mixture 2 base noadapt split2
tools/ab.sh sift1m latent 2 base noadapt split2
BENCH_ARGS="--scaling strong --nq 1250" tools/ab.sh sift1m mixture 2 base noadapt split2
