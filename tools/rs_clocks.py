"""Per-phase cycle split of k_screen_r (timing experiment; needs a -DRS_CLOCKS
variant library):  VARIANT_FLAGS=-DRS_CLOCKS tools/build_variant.sh lira_rscreen.hip \
    lira-ann-search_amd/csrc/lira_rscreen.hip rclk
  LIRA_HIP_LIB=variants/rclk.so python tools/rs_clocks.py <config> <data> [option=value ...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lira-ann-search_amd"))
import torch  # noqa: E402

from lira_amd import PartitionedIndex, rank_nearest, _lib  # noqa: E402
from lira_amd.synthetic import CONFIGS, workload  # noqa: E402

cfg, data = sys.argv[1], sys.argv[2]
opts = dict((a.split("=")[0], int(a.split("=")[1])) for a in sys.argv[3:])
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
nq = int(os.environ.get("NQ", nq))
dev = torch.device("cuda", 0)
x, c, assign, mq = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0, **opts).build(assign[:, None] if assign.dim() == 1 else assign, x, B)
q = mq(nq, 1335)
probe = rank_nearest(q, c, nprobe)
lib = _lib.load()
v = (ctypes.c_uint64 * 16)()
for _ in range(3):
    idx.search(q, probe, k)
torch.cuda.synchronize()
lib.lira_debug_rs_clocks(v)
idx.set_profiling(True)
reps = 5
for _ in range(reps):
    idx.search(q, probe, k)
torch.cuda.synchronize()
lib.lira_debug_rs_clocks(v)
pr = idx.profile_read()
items, entries = v[7] & 0xffffffff, v[7] >> 32
skipped, mdrains = v[9] & 0xffffffff, v[9] >> 32
v[7], v[9] = items, skipped
names = ["prologue", "first-tile", "thresholds", "mfma+loads", "passbits", "queue", "epilogue"]
waves = max(1, v[10])
tot = sum(v[i] for i in range(7))
print(cfg, data, opts, idx.describe(nq, nprobe, k))
print("scan_ms %.3f per call; items %d tiles %d skipped %d per call; waves %d" % (
    pr["scan_ms"] / reps, v[7] / reps, v[8] / reps, v[9] / reps, waves / reps))
print("per wave per call (cycles): " + "  ".join("%s %.0f (%.2f)" % (n, v[i] / waves, v[i] / max(1, tot))
                                                   for i, n in enumerate(names)))
t = max(1, v[8])
print("per tile (cycles): " + "  ".join("%s %.0f" % (n, v[i] / t) for i, n in zip((2, 3, 4, 5), names[2:6])))
print("per tile: survivors %.2f  entries with survivors %.2f  mid-selection drains %.3f  list flushes %.3f" % (
    v[11] / t, entries / t, mdrains / t, v[12] / t))
print("group 0 (nearest partition): tiles %.3f of all, survivors %.3f of all (%.2f per tile; others %.2f per tile)" % (
    v[14] / t, v[13] / max(1, v[11]), v[13] / max(1, v[14]), (v[11] - v[13]) / max(1, t - v[14])))
