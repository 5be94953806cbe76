"""Per-phase cycle split of k_screen_v (a -DLIRA_VCLOCKS build:
VARIANT_FLAGS=-DLIRA_VCLOCKS tools/build_variant.sh lira_vscreen.hip
lira-ann-search_amd/csrc/lira_vscreen.hip vclk; LIRA_HIP_LIB=variants/vclk.so):
wave 0 of every workgroup adds its clock64() deltas per phase.

usage: python tools/vclocks.py <config> <data> [nq] [option=value ...]
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
opts.setdefault("wide", 2)
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
keys = ("chunks_computed", "chunks_nominal", "blocks", "blocks_dropped", "blocks_skipped", "rechecked", "rescans",
        "survivors")
v = [st[kk] for kk in keys]
names = ["-", "prologue", "refresh", "mfma issue", "selection", "issue+skip", "epilogue", "claims"]
print(cfg, data, nq, opts, idx.describe(nq, nprobe, k))
print("scan_ms %.3f plan_ms %.3f merge_ms %.3f" % (pr["scan_ms"] / pr["calls"], pr["plan_ms"] / pr["calls"],
                                                   pr["merge_ms"] / pr["calls"]))
tot = max(1, sum(v[1:8]))
nw = 2 * 256  # wave 0 of each workgroup (2 per CU)
print("per wave-0 (%d waves): " % nw + "  ".join("%s %.3g (%.2f)" % (n, x / nw, x / tot)
                                                for n, x in zip(names[1:8], v[1:8])))
