"""Per-phase cycle split of k_screen_w (a -DLIRA_WCLOCKS build, e.g.
VARIANT_FLAGS=-DLIRA_WCLOCKS tools/build_variant.sh lira_wscreen.hip
lira-ann-search_amd/csrc/lira_wscreen.hip wclk; LIRA_HIP_LIB=variants/wclk.so):
wave 0's loop split and the scheduling wave's decide time, per workgroup-block.

usage: python tools/wclocks.py <config> <data> [nq] [option=value ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lira-ann-search_amd"))
import torch  # noqa: E402

from lira_amd import PartitionedIndex, rank_nearest  # noqa: E402
from lira_amd.synthetic import CONFIGS, workload  # noqa: E402

cfg, data = sys.argv[1], sys.argv[2]
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
rest = sys.argv[3:]
if rest and "=" not in rest[0]:
    nq = int(rest.pop(0))
opts = dict((a.split("=")[0], int(a.split("=")[1])) for a in rest)
dev = torch.device("cuda", 0)
x, c, assign, mq = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0, **opts).build(assign[:, None] if assign.dim() == 1 else assign, x, B)
q = mq(nq, 1335)
probe = rank_nearest(q, c, nprobe)
for _ in range(3):
    idx.search(q, probe, k)
idx.set_profiling(True)
for _ in range(5):
    idx.search(q, probe, k)
pr = idx.profile_read()
idx.set_profiling(False)
idx.set_stats(True)
idx.search(q, probe, k)
st = idx.stats_read()
idx.set_stats(False)
names = ["loop", "wait+barrier", "issue", "transitions", "refresh", "mfma", "select", "decide(SW)"]
v = [st[kk] for kk in ("chunks_computed", "chunks_nominal", "blocks", "blocks_dropped", "blocks_skipped",
                         "rechecked", "rescans", "survivors")]
print(cfg, data, nq, opts, idx.describe(nq, nprobe, k))
print("scan_ms %.3f plan_ms %.3f merge_ms %.3f" % (pr["scan_ms"] / pr["calls"], pr["plan_ms"] / pr["calls"],
                                                   pr["merge_ms"] / pr["calls"]))
tot = max(1, v[0])
print("  ".join("%s %.3g (%.2f)" % (n, x, x / tot) for n, x in zip(names, v)))
