#!/bin/bash
# On the GPU box: L2 hit rate of the scan kernel (TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)),
# one PMC pass of its own: tools/l2_hits.sh <config> <data>
set -euo pipefail
CFG=$1; DATA=$2
OUT=gpurun_out/l2_${CFG}_${DATA}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT -o run --output-format csv -- \
    python3 bench.py --config $CFG --data $DATA --no-cpu-baseline --no-exact --no-pipeline --contrast none \
    --recall-sample 4 --steps 3 --warmup 1 > $OUT/run.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    name = r.get("Kernel_Name", "")
    if "k_screen" not in name:
        continue
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    h, m = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
    print(k[:60], "L2 hit rate %.3f" % (h / max(1.0, h + m)), "hits", int(h), "misses", int(m))
PY
