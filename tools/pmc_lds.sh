#!/bin/bash
# One PMC pass (LDS counters) of the bench per variant ("base" = in-tree .so):
#   bash tools/pmc_lds.sh <config> <data> name1 name2 ...  -> per-kernel medians via tools/pmc_kstats.py
set -euo pipefail
export TMPDIR=/tmp
cfg=$1; data=$2; shift 2
for v in "$@"; do
  lib=variants/$v.so; [ "$v" = base ] && lib=lira-ann-search_amd/lira_amd/liblira_hip.so
  out=gpurun_out/pl_${v}_${cfg}_${data}
  mkdir -p $out
  LIRA_HIP_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-trace \
      -d $out -o run --output-format csv -- python3 bench.py --config $cfg --data $data --steps 3 --warmup 1 \
      --no-cpu-baseline --no-exact --no-pipeline --contrast none --recall-sample 4 > $out/log.txt 2>&1
  echo "== $v $cfg $data"
  python3 tools/pmc_kstats.py $out
done
