#!/bin/bash
# On the GPU box: rocprof evidence for each config (tools/profile_box.sh), then
# the default bench with its CPU baseline.  usage: tools/profile_all.sh <tag> cfg...
set -euo pipefail
TAG=$1; shift
for cfg in "$@"; do
  bash tools/profile_box.sh "${TAG}_$cfg" --config "$cfg" > /dev/null
  echo "profiled $cfg"
done
