#!/bin/bash
set -e
tools/ab.sh gist1m mixture 1 base unfused
tools/ab.sh gist1m latent 1 base unfused
grep -o '"kernels_ms_per_step": {[^}]*}' gpurun_out/ab_base.log
