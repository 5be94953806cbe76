#!/bin/bash
# Same-box A/B of index options on the in-tree library:
#   tools/ab_opts.sh <config> <data> "<opts A>" "<opts B>" ...   (each: space-separated name=value, or "-")
# (extra bench args via BENCH_ARGS)
cfg=$1; data=$2; shift 2
mkdir -p gpurun_out
i=0
for o in "$@"; do
  i=$((i+1))
  args=""; [ "$o" != "-" ] && for kv in $o; do args="$args --opt $kv"; done
  timeout -k 10 240 python bench.py --config "$cfg" --data "$data" --steps 20 --warmup 3 \
      --no-cpu-baseline --no-exact --no-pipeline --contrast none $args $BENCH_ARGS > gpurun_out/abo_$i.log 2>&1 || { echo "opts [$o] failed"; tail -5 gpurun_out/abo_$i.log; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/abo_$i.log').read().strip().splitlines()[-1]); k=j['kernels_ms_per_step']; \
print('$cfg/$data', '[$o]', 'qps %.0f step %.3f scan %.3f merge %.3f plan %.3f rank %.3f exact %s' % (j['value'], j['ms_per_step'], k['scan'], k['merge'], k['plan'], k.get('rank_nearest',0), j['parity_bit_exact']))" \
      | tee -a gpurun_out/abo.txt
done
