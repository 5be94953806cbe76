#!/bin/bash
# same-box A/B of variants on SIFT1M latent + mixture: tools/r4_ab.sh <rounds> v1 v2 ...
set -e
r=$1; shift
tools/ab.sh sift1m latent $r "$@"
tools/ab.sh sift1m mixture $r "$@"
