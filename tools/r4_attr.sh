#!/bin/bash
set -e
mkdir -p gpurun_out
tools/ab.sh sift1m latent 1 base nosurv nodrain noepi same
tools/ab.sh sift1m mixture 1 base nosurv nodrain noepi same
tools/pmc_ab.sh sift1m latent base nosurv
