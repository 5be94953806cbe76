#!/bin/bash
# rocprofv3 kernel trace of the bench for variants/<name>.so ("base" = in-tree):
#   bash tools/trace_ab.sh <config> <data> name1 name2 ...
set -euo pipefail
export TMPDIR=/tmp
cfg=$1; data=$2; shift 2
for v in "$@"; do
  lib=variants/$v.so; [ "$v" = base ] && lib=lira-ann-search_amd/lira_amd/liblira_hip.so
  out=gpurun_out/tr_${v}_${cfg}_${data}
  mkdir -p $out
  LIRA_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- \
      python3 bench.py --config $cfg --data $data --steps 10 --warmup 2 --no-cpu-baseline --no-exact --no-pipeline \
      --contrast none --recall-sample 4 > $out/log.txt 2>&1
done
