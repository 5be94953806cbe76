#!/bin/bash
# On the GPU box: rocprof evidence for configs x distributions
# (tools/profile_box.sh).  usage: tools/profile_all.sh <tag> cfg:data[:passes] ...
set -euo pipefail
TAG=$1; shift
for spec in "$@"; do
  IFS=: read -r cfg data passes <<< "$spec"
  bash tools/profile_box.sh "$TAG" "$cfg" "$data" "${passes:-all}" > /dev/null
  echo "profiled $cfg/$data"
done
