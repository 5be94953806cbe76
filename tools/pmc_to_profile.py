"""Turn a tools/profile_box.sh summary into the per-(config, data) record
bench.py reads (profiles/pmc_scan_<config>_<data>.json) and copy the evidence
into profiles/.  The record names the scan kernel and plan (lira_scan_describe,
from the profiled bench's own JSON line) and the batch size, so bench.py uses
it only for the same kernel on the same shape.

usage: python tools/pmc_to_profile.py <config> <data> <gpurun_out/prof_DIR> <round tag, e.g. r02>
"""
import json
import os
import shutil
import sys

WORKLOADS = {
    "sift1m": "sift1m (N=1M d=128 B=64 nprobe=8 k=10 L2, 10k queries)",
    "gist1m": "gist1m (N=1M d=960 B=128 nprobe=16 k=10 L2, 1k queries)",
    "deep10m": "deep10m (N=10M d=96 B=256 nprobe=32 k=100 IP, 10k queries)",
    "bigann100m": "bigann100m (N=100M n_mul=2 d=128 B=1024 nprobe=32 k=10 L2, 10k queries)",
}


def bench_line(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return {}


def main(cfg, data, src, tag):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    summ = json.load(open(os.path.join(src, "summary.json")))
    bl = bench_line(os.path.join(src, "trace.log"))
    # the default path's scan kernel (screened: k_screen_m / k_screen), else the
    # all-exact k_scan; the one with the most total time
    scan = [(k, v) for k, v in summ.items() if k.startswith("lira::k_screen")] or \
           [(k, v) for k, v in summ.items() if k.startswith("lira::k_scan")]
    if not scan:
        raise SystemExit("no scan kernel entry in summary")
    tot = lambda kv: kv[1].get("trace", {}).get("calls", 0) * (kv[1].get("trace", {}).get("avg_ns") or 0)  # noqa: E731
    name, e = max(scan, key=tot)
    p = e.get("pmc", {})
    rec = {
        "kernel": name,
        "kernel_desc": bl.get("kernel"),
        "nq": (bl.get("config") or {}).get("queries_per_rank"),
        "workload": WORKLOADS.get(cfg, cfg) + f", {data} data",
        "hbm_bytes_per_launch": e.get("hbm_bytes_per_launch"),
        "avg_ns_trace": e.get("trace", {}).get("avg_ns"),
        "bench_kernel_ms": ((bl.get("roofline") or {}).get("kernel_ms")),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with "
                  "--kernel-trace; bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE "
                  "counts half of 16-B/lane streaming reads incl. LDS-DMA loads, "
                  "MI355X_MICROARCH.md HBM section)",
        "FETCH_SIZE_KiB": p.get("FETCH_SIZE"),
        "WRITE_SIZE_KiB": p.get("WRITE_SIZE"),
        "mfma_busy_pct": e.get("mfma_busy_pct"),
        "valu_busy_pct": e.get("valu_busy_pct"),
        "wave_cycle_split": e.get("wave_cycle_split"),
        "lds_bank_conflicts": p.get("SQ_LDS_BANK_CONFLICT"),
        "source": f"profiles/{tag}_{cfg}_{data}_pmc_summary.json",
    }
    # median launch of that kernel in the trace: the average also holds the
    # bench's one work-counter launch (stats on: per-block atomics, ~7x slower)
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        import csv
        short = name.split("(")[0]
        ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tr))
                    if r["Kernel_Name"].split("(")[0].replace("void ", "") == short)
        if ds:
            rec["median_ns_trace"] = ds[len(ds) // 2]
            rec["launches_trace"] = len(ds)
            rec["note_trace"] = ("avg_ns_trace includes the bench's single stats-on launch (work counters, "
                                 "atomics per block); median_ns_trace is the timed launches' figure")
    out = os.path.join(root, "profiles")
    json.dump(rec, open(os.path.join(out, f"pmc_scan_{cfg}_{data}.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, "summary.json"), os.path.join(out, f"{tag}_{cfg}_{data}_pmc_summary.json"))
    st = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(out, f"{tag}_{cfg}_{data}_kernel_stats.csv"))
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
