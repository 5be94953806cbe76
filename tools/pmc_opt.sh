#!/bin/bash
# Same-box PMC comparison of index-option variants (bench.py --opt):
#   tools/pmc_opt.sh <config> <data> "<opts1>" "<opts2>" ...   (opts: space-separated name=value; "" = defaults)
# -> gpurun_out/pmcopt_<i>/summary.json (FETCH_SIZE, TCC hit/miss, SQ busy/wait/MFMA counters per kernel)
set -euo pipefail
cfg=$1; data=$2; shift 2
export TMPDIR=/tmp
i=0
for opts in "$@"; do
  OUT=gpurun_out/pmcopt_$i
  rm -rf $OUT; mkdir -p $OUT
  echo "$opts" > $OUT/opts.txt
  args=""
  for o in $opts; do args="$args --opt $o"; done
  B="python3 bench.py --config $cfg --data $data --no-cpu-baseline --no-exact --no-pipeline --contrast none --recall-sample 4 --steps 3 --warmup 1 $args"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/tcc -o run --output-format csv -- $B > $OUT/tcc.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq1 -o run --output-format csv -- $B > $OUT/sq1.log 2>&1
  python3 tools/pmc_summary.py $OUT > $OUT/summary.json
  i=$((i+1))
done
