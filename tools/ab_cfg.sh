#!/bin/bash
# Same-box A/B over configs x distributions with index options:
#   tools/ab_cfg.sh "<opts>" cfg:data ...   (opts: space-separated name=value, may be empty)
opts=$1; shift
mkdir -p gpurun_out
args=""
for o in $opts; do args="$args --opt $o"; done
for spec in "$@"; do
  cfg=${spec%%:*}; data=${spec#*:}
  timeout -k 10 200 python bench.py --config $cfg --data $data --steps 20 --warmup 3 --no-cpu-baseline --no-pipeline \
      --no-exact --contrast none $args > gpurun_out/abcfg.json 2> gpurun_out/abcfg.err || { echo "$spec failed"; tail -5 gpurun_out/abcfg.err; exit 1; }
  python3 -c "import json; j=json.loads(open('gpurun_out/abcfg.json').read().strip().splitlines()[-1]); k=j['kernels_ms_per_step']; w=j['roofline']['work']; \
print('$spec [$opts]', 'qps %.0f scan %.3f merge %.3f plan %.3f exact %s surv %d rechk/q %.1f' % (j['value'], k['scan'], k['merge'], k['plan'], j['parity_bit_exact'], w['survivors'], w['rechecked_per_query']))" | tee -a gpurun_out/ab.txt
done
