#!/bin/bash
# Same-box PMC comparison of variants/<name>.so ("base" = in-tree .so):
#   tools/pmc_ab.sh <config> <data> name1 name2 ...   -> gpurun_out/pmcab_<name>/summary.json
set -euo pipefail
cfg=$1; data=$2; shift 2
export TMPDIR=/tmp
for v in "$@"; do
  OUT=gpurun_out/pmcab_$v
  mkdir -p $OUT
  B="python3 bench.py --config $cfg --data $data --no-cpu-baseline --no-exact --no-pipeline --contrast none --recall-sample 4 --steps 3 --warmup 1"
  lib=variants/$v.so; [ "$v" = base ] && lib=lira-ann-search_amd/lira_amd/liblira_hip.so
  export LIRA_HIP_LIB=$lib
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq1 -o run --output-format csv -- $B > $OUT/sq1.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU --kernel-trace -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
  python3 tools/pmc_summary.py $OUT > $OUT/summary.json
done
