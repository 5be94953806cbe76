"""Summarise rocprofv3 CSVs of tools/profile_box.sh per lira kernel.

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB: on gfx950
FETCH_SIZE counts exactly half of a wide coalesced streaming read
(MI355X_MICROARCH.md, HBM section), and the scan's tile loads are 16 B/lane
coalesced; WRITE_SIZE is exact for 16-B stores and near-exact otherwise.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


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
            acc[k]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        for k, cs in acc.items():
            e = out.setdefault(k, {}).setdefault("pmc", {})
            for c, v in cs.items():
                if c == "_dur_ns":
                    continue
                e[c] = sum(v) / len(v)
    for k, e in out.items():
        p = e.get("pmc", {})
        if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
            e["hbm_bytes_per_launch"] = (2 * p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024
        if "FETCH_SIZE" in p:
            e["l2_miss_read_bytes_per_launch"] = 2 * p["FETCH_SIZE"] * 1024
        if "TCC_HIT_sum" in p and "TCC_MISS_sum" in p and p["TCC_HIT_sum"] + p["TCC_MISS_sum"]:
            e["l2_hit_rate"] = p["TCC_HIT_sum"] / (p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
        if "SQ_ACTIVE_INST_VALU" in p and "GRBM_GUI_ACTIVE" in p and p["GRBM_GUI_ACTIVE"]:
            # VALUBusy as rocprof defines it: 100*sum(ACTIVE_INST_VALU)/CU_NUM/GRBM_GUI_ACTIVE
            # (ACTIVE_INST_VALU in quad-cycles; GRBM summed over 8 XCDs)
            e["valu_busy_pct"] = 100 * p["SQ_ACTIVE_INST_VALU"] * 4 / 256 / (p["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in p and "GRBM_GUI_ACTIVE" in p and p["GRBM_GUI_ACTIVE"]:
            # MFMA busy cycles (summed over SIMDs) per SIMD-cycle of the kernel
            e["mfma_busy_pct"] = 100 * p["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4) / (p["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_WAVE_CYCLES" in p and p["SQ_WAVE_CYCLES"]:
            w = p["SQ_WAVE_CYCLES"]
            e["wave_cycle_split"] = {
                "active_inst_any": p.get("SQ_ACTIVE_INST_ANY", 0) / w,
                "wait_any": p.get("SQ_WAIT_ANY", 0) / w,
                "wait_inst_any": p.get("SQ_WAIT_INST_ANY", 0) / w}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
