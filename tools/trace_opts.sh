#!/bin/bash
# rocprofv3 kernel-trace stats of the bench for one library and several option sets:
#   bash tools/trace_opts.sh <lib name|base> <config> <data> "<opts1>" "<opts2>" ...
#   (opts: space-separated name=value, "" = defaults; BENCH_ARGS: extra bench args)
# -> gpurun_out/to_<lib>_<cfg>_<data>_<i>/run_kernel_stats.csv, summarised by tools/kstats.py
set -euo pipefail
export TMPDIR=/tmp
v=$1; cfg=$2; data=$3; shift 3
lib=variants/$v.so; [ "$v" = base ] && lib=lira-ann-search_amd/lira_amd/liblira_hip.so
i=0
for opts in "$@"; do
  args=""
  for o in $opts; do args="$args --opt $o"; done
  out=gpurun_out/to_${v}_${cfg}_${data}_$i
  mkdir -p $out
  LIRA_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- \
      python3 bench.py --config $cfg --data $data --steps 10 --warmup 2 --no-cpu-baseline --no-exact --no-pipeline \
      --contrast none --recall-sample 4 $args $BENCH_ARGS > $out/log.txt 2>&1
  echo "== $v $cfg $data [$opts]"
  python3 tools/kstats.py $out
  i=$((i+1))
done
