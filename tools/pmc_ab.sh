#!/bin/bash
# Same-box PMC comparison of variants/<name>.so on one config:
#   tools/pmc_ab.sh <config> name1 name2 ...   -> gpurun_out/pmcab_<name>/summary.json
set -euo pipefail
cfg=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  OUT=gpurun_out/pmcab_$v
  mkdir -p $OUT
  B="python3 bench.py --config $cfg --no-cpu-baseline --recall-sample 4 --steps 3 --warmup 1"
  export LIRA_HIP_LIB=variants/$v.so
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq1 -o run --output-format csv -- $B > $OUT/sq1.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU --kernel-trace -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1
  python3 tools/pmc_summary.py $OUT > $OUT/summary.json
done
