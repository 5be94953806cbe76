#!/bin/bash
# rocprofv3 kernel trace of the MLP-probed pipeline (tools/pipeline_prof.py), with
# and without the probes hint:  bash tools/prof_pipeline.sh <config> <data>
set -euo pipefail
export TMPDIR=/tmp
cfg=${1:-sift1m}; data=${2:-mixture}
for hint in 0 8; do
  out=gpurun_out/pipe_${cfg}_${data}_h$hint
  mkdir -p $out
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- \
      python3 tools/pipeline_prof.py $cfg $data 64 10 $hint > $out/log.txt 2>&1
  echo "hint $hint: $(tail -1 $out/log.txt)"
done
