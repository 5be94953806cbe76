"""Per-kernel median durations (us) of a rocprofv3 kernel trace directory (the
library's own kernels), from *_kernel_trace.csv: usage python3 tools/kstats.py <dir>"""
import csv
import glob
import statistics
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = {}
for r in rows:
    n = r["Kernel_Name"]
    if "lira::" not in n:
        continue
    n = n.replace("void ", "").replace("lira::", "").split("(")[0]
    by.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for n, v in sorted(by.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    if len(v) >= 5:
        print(f"  {n:60s} n={len(v):4d} median {statistics.median(v):8.2f} us  min {min(v):8.2f}")
