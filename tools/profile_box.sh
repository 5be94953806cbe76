#!/bin/bash
# Run on the GPU box (via gpurun) from the repo root:  bash tools/profile_box.sh <tag> [bench args]
# rocprofv3 kernel-trace/stats of the bench, then separate PMC passes (one
# counter group each, never combined with runtime/sys traces), summarised by
# tools/pmc_summary.py into gpurun_out/prof_<tag>/summary.json.
set -euo pipefail
TAG=${1:-r01}
shift || true
ARGS="$@"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --contrast none --recall-sample 4 $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B --steps 10 --warmup 2 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq1 -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU --kernel-trace -d $OUT/sq2 -o run --output-format csv -- $B --steps 3 --warmup 1 > $OUT/sq2.log 2>&1
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
