"""Per-kernel medians of each PMC counter in a rocprofv3 --pmc output directory
(the library's own kernels): python3 tools/pmc_kstats.py <dir>"""
import csv
import glob
import statistics
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = {}
for r in rows:
    n = r["Kernel_Name"]
    if "lira::" not in n:
        continue
    n = n.replace("void ", "").replace("lira::", "").split("(")[0]
    key = (n, r["Counter_Name"])
    by.setdefault(key, {}).setdefault(r["Dispatch_Id"], 0.0)
    by[key][r["Dispatch_Id"]] += float(r["Counter_Value"])
for (n, c), d in sorted(by.items()):
    v = list(d.values())
    print(f"  {n:40s} {c:24s} n={len(v):3d} median {statistics.median(v):14.0f}")
