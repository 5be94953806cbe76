#!/bin/bash
# Same-box sweep: tools/ab_env.sh <config> <variant> VAR v1 v2 ...  (bench per value of env VAR)
cfg=$1; v=$2; var=$3; shift 3
mkdir -p gpurun_out
for val in "$@"; do
  env "$var=$val" LIRA_HIP_LIB=variants/$v.so timeout -k 10 150 python bench.py --config "$cfg" --steps 20 --warmup 3 \
      --no-cpu-baseline > gpurun_out/abenv.log 2>&1 || { echo "$v $var=$val failed"; tail -5 gpurun_out/abenv.log; exit 1; }
  python3 -c "import json; j=json.loads(open('gpurun_out/abenv.log').read().strip().splitlines()[-1]); \
print('$cfg $v $var=$val', 'qps %.0f scan_ms %.3f merge_ms %.3f exact %s' % (j['value'], j['kernels_ms_per_step']['scan'], j['kernels_ms_per_step']['merge'], j['parity_bit_exact']))" | tee -a gpurun_out/ab.txt
done
