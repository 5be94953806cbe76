#!/bin/bash
# Same-box A/B of variants/<name>.so: tools/ab.sh <config> <rounds> name1 name2 ...
cfg=$1; rounds=$2; shift 2
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for v in "$@"; do
    LIRA_HIP_LIB=variants/$v.so timeout -k 10 150 python bench.py --config "$cfg" --steps 20 --warmup 3 \
        --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); \
print('$cfg', '$v', 'round', $r, 'qps %.0f scan_ms %.3f exact %s' % (j['value'], j['kernels_ms_per_step']['scan'], j['parity_bit_exact']))" \
        | tee -a gpurun_out/ab.txt
  done
done
