#!/bin/bash
# Run on the GPU box (via gpurun) from the repo root:
#   bash tools/profile_box.sh <tag> <config> <data> [passes] [extra bench args]
# rocprofv3 kernel-trace/stats of the bench, then separate PMC passes (one
# counter group each, never combined with runtime/sys traces), summarised by
# tools/pmc_summary.py and turned into profiles/pmc_scan_<config>_<data>.json
# by tools/pmc_to_profile.py (the record bench.py reads for roofline.traffic).
# passes: "all" (trace fetch write sq1 sq2, default) or "mem" (trace fetch write).
set -euo pipefail
TAG=${1:-r02}
CFG=${2:-sift1m}
DATA=${3:-mixture}
PASSES=${4:-all}
shift 4 || shift $#
ARGS="$@"
OUT=gpurun_out/prof_${TAG}_${CFG}_${DATA}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --config $CFG --data $DATA --no-cpu-baseline --no-exact --no-pipeline --contrast none --recall-sample 4 $ARGS"
T=${PROF_TIMEOUT:-240}
timeout -k 10 $T rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B --steps 10 --warmup 2 > $OUT/trace.log 2>&1
timeout -s KILL $T rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/fetch.log 2>&1
timeout -s KILL $T rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/write.log 2>&1
if [ "$PASSES" = "all" ]; then
timeout -s KILL $T rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq1 -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/sq1.log 2>&1
timeout -s KILL $T rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU --kernel-trace -d $OUT/sq2 -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/sq2.log 2>&1
fi
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
python3 tools/pmc_to_profile.py $CFG $DATA $OUT $TAG
