#!/bin/bash
set -e
rm -f gpurun_out/ab.txt
BENCH_ARGS="" tools/ab.sh gist1m mixture 3 base prev
tools/ab.sh gist1m latent 2 base prev
