#!/bin/bash
# Same-box A/B of variants/<name>.so (tools/build_variant.sh), "base" = the in-tree .so:
#   tools/ab.sh <config> <data> <rounds> name1 name2 ...   (extra bench args via BENCH_ARGS)
cfg=$1; data=$2; rounds=$3; shift 3
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for v in "$@"; do
    lib=variants/$v.so; [ "$v" = base ] && lib=lira-ann-search_amd/lira_amd/liblira_hip.so
    LIRA_HIP_LIB=$lib timeout -k 10 200 python bench.py --config "$cfg" --data "$data" --steps 20 --warmup 3 \
        --no-cpu-baseline --no-exact --no-pipeline --contrast none $BENCH_ARGS > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); k=j['kernels_ms_per_step']; \
print('$cfg/$data', '$v', 'round', $r, 'qps %.0f scan %.3f merge %.3f plan %.3f exact %s' % (j['value'], k['scan'], k['merge'], k['plan'], j['parity_bit_exact']))" \
        | tee -a gpurun_out/ab.txt
  done
done
