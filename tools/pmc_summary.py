"""Summarise rocprofv3 CSVs of tools/profile_box.sh per lira kernel.

Per counter the MEDIAN over the kernel's launches is kept (the bench's one
stats-on launch, with per-block atomics, is an outlier both in time and in
bytes; a mean would carry it into every per-launch figure).

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB: on gfx950
FETCH_SIZE counts exactly half of a wide coalesced streaming read
(MI355X_MICROARCH.md, HBM section), and the scan's tile loads are 16 B/lane
coalesced; WRITE_SIZE is exact for 16-B stores and near-exact otherwise.

Utilisation is normalised by the kernel's median duration in the plain
kernel trace (no counters: PMC passes serialise dispatches and stretch them)
at the 2.4 GHz peak clock, over the chip's 1024 SIMDs -- so it is a lower
bound when the chip runs below 2.4 GHz, and never above 100 %:
  mfma_busy_pct  = SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe cycles summed over
                   SIMDs; checked on k_centroid_gemm: 40 k v_mfma_f32_32x32x2_f32
                   x 64 cycles = 2.56 M against 2.57 M counted) / SIMD-cycles
  valu_issue_pct = SQ_INSTS_VALU x 2 cycles (one wave64 VALU instruction per 2
                   SIMD cycles at full rate; MFMA instructions included) / SIMD-cycles
(round 2's valu_busy_pct summed SQ_ACTIVE_INST_VALU over co-resident waves and
divided by GRBM_GUI_ACTIVE, which is why it read above 100 %).
"""
import csv
import json
import os
import sys
from collections import defaultdict

CLOCK_GHZ = 2.4
SIMDS = 1024


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main(d):
    out = {}
    st = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            if "lira::" in r["Name"]:
                out.setdefault(short(r["Name"]), {})["trace"] = {
                    "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                    "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                    "pct": float(r["Percentage"])}
    tr = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        durs = defaultdict(list)
        for r in csv.DictReader(open(tr)):
            if "lira::" in r["Kernel_Name"]:
                durs[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in durs.items():
            out.setdefault(k, {}).setdefault("trace", {})["median_ns"] = median(v)
    for sub in ("fetch", "write", "sq1", "sq2", "tcc"):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        acc = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(f)):
            if "lira::" not in r["Kernel_Name"]:
                continue
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            e = out.setdefault(k, {}).setdefault("pmc", {})
            for c, v in cs.items():
                e[c] = median(v)
                e.setdefault("_launches", {})[c] = len(v)
    for k, e in out.items():
        p = e.get("pmc", {})
        if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
            e["hbm_bytes_per_launch"] = (2 * p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024
        if "FETCH_SIZE" in p:
            e["l2_miss_read_bytes_per_launch"] = 2 * p["FETCH_SIZE"] * 1024
        if "TCC_HIT_sum" in p and "TCC_MISS_sum" in p and p["TCC_HIT_sum"] + p["TCC_MISS_sum"]:
            e["l2_hit_rate"] = p["TCC_HIT_sum"] / (p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
        dur = (e.get("trace") or {}).get("median_ns")
        if dur:
            simd_cycles = SIMDS * dur * CLOCK_GHZ
            if "SQ_VALU_MFMA_BUSY_CYCLES" in p:
                e["mfma_busy_pct"] = min(100.0, 100 * p["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles)
            if "SQ_INSTS_VALU" in p:
                e["valu_issue_pct"] = min(100.0, 100 * p["SQ_INSTS_VALU"] * 2 / simd_cycles)
            e["utilisation_basis"] = (f"median trace duration {dur} ns x {CLOCK_GHZ} GHz x {SIMDS} SIMDs "
                                      "(lower bound below peak clock)")
        if "SQ_WAVE_CYCLES" in p and p["SQ_WAVE_CYCLES"]:
            w = p["SQ_WAVE_CYCLES"]
            e["wave_cycle_split"] = {
                "active_inst_any": p.get("SQ_ACTIVE_INST_ANY", 0) / w,
                "wait_any": p.get("SQ_WAIT_ANY", 0) / w,
                "wait_inst_any": p.get("SQ_WAIT_INST_ANY", 0) / w}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
