#!/bin/bash
# Same-box sweep of one index option (include/lira_hip.h LIRA_OPT_*):
#   tools/ab_env.sh <config> <data> <option> v1 v2 ...
cfg=$1; data=$2; opt=$3; shift 3
mkdir -p gpurun_out
for val in "$@"; do
  timeout -k 10 200 python bench.py --config "$cfg" --data "$data" --steps 20 --warmup 3 --no-cpu-baseline --no-pipeline \
      --no-exact --contrast none --opt "$opt=$val" $BENCH_ARGS > gpurun_out/abenv.log 2>&1 || { echo "$opt=$val failed"; tail -5 gpurun_out/abenv.log; exit 1; }
  python3 -c "import json; j=json.loads(open('gpurun_out/abenv.log').read().strip().splitlines()[-1]); k=j['kernels_ms_per_step']; \
print('$cfg/$data $opt=$val', 'qps %.0f scan %.3f merge %.3f plan %.3f exact %s' % (j['value'], k['scan'], k['merge'], k['plan'], j['parity_bit_exact']))" | tee -a gpurun_out/ab.txt
done
