#!/bin/bash
# On the GPU box: the round's bench lines, one JSON line each into gpurun_out/<tag>_bench_<name>.json
#   bash tools/bench_all.sh <tag> name:args ...   e.g. r06 "sift:" "sift_uniform:--data uniform --contrast none"
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  echo "== $name: bench.py $args"
  timeout -k 10 900 python3 -u bench.py $args > gpurun_out/${TAG}_bench_${name}.out 2> gpurun_out/${TAG}_bench_${name}.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "bench $name failed rc=$rc"; tail -5 gpurun_out/${TAG}_bench_${name}.err; exit $rc; fi
  tail -1 gpurun_out/${TAG}_bench_${name}.out > gpurun_out/${TAG}_bench_${name}.json
  python3 -c "import json; j=json.load(open('gpurun_out/${TAG}_bench_${name}.json')); print('$name', 'value %.0f' % j['value'], 'ms/step %.4f' % j['ms_per_step'], 'exact', j.get('parity_bit_exact'), 'frac', round(j['roofline']['frac'], 3), j['roofline']['binding'], 'traffic', j['roofline']['traffic'])"
done
