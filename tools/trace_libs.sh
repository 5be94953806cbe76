#!/bin/bash
# rocprofv3 kernel-trace medians of the bench for several libraries (same options):
#   bash tools/trace_libs.sh <config> <data> name1 name2 ...   ("base" = in-tree; BENCH_ARGS: extra args)
set -euo pipefail
export TMPDIR=/tmp
cfg=$1; data=$2; shift 2
for v in "$@"; do
  lib=variants/$v.so; [ "$v" = base ] && lib=lira-ann-search_amd/lira_amd/liblira_hip.so
  out=gpurun_out/tl_${v}_${cfg}_${data}
  mkdir -p $out
  LIRA_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- \
      python3 bench.py --config $cfg --data $data --steps 10 --warmup 2 --no-cpu-baseline --no-exact --no-pipeline \
      --contrast none --recall-sample 4 ${BENCH_ARGS:-} > $out/log.txt 2>&1
  echo "== $v $cfg $data ${BENCH_ARGS:-}"
  python3 tools/kstats.py $out
done
