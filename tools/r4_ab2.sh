#!/bin/bash
# same-box A/B: GIST1M seed tiles, SIFT1M prescan; then BIGANN-100M lines at HEAD (latent with the r04 PMC record)
set -e
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
rm -f gpurun_out/abo.txt
tools/ab_opts.sh gist1m latent seed_tiles=2 seed_tiles=1 seed_tiles=2 seed_tiles=1
tools/ab_opts.sh gist1m mixture seed_tiles=2 seed_tiles=1
tools/ab_opts.sh sift1m mixture - rescan=1 - rescan=1
tools/ab_opts.sh sift1m latent - rescan=1
timeout -k 10 900 python bench.py --config bigann100m --data latent --steps 5 --warmup 2 > gpurun_out/bench_bigann_latent.log 2>gpurun_out/bench_bigann_latent.err || { tail -5 gpurun_out/bench_bigann_latent.err; exit 1; }
echo latent done
timeout -k 10 900 python bench.py --config bigann100m --data mixture --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_bigann_mixture.log 2>gpurun_out/bench_bigann_mixture.err || { tail -5 gpurun_out/bench_bigann_mixture.err; exit 1; }
echo mixture done
