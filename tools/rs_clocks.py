"""Phase split of k_screen_r (timing experiment; clock64 stamps need an lgkmcnt(0)
each, so the variant runs slower: shares only).  Build the variant from a copy of
lira_rscreen.hip with g_rs_clk stamps (tools/build_variant.sh lira_rscreen.hip <src> rsclk).
usage: LIRA_HIP_LIB=variants/rsclk.so python tools/rs_clocks.py [config] [data] [opt=value ...]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lira-ann-search_amd"))
from lira_amd import PartitionedIndex, rank_nearest  # noqa: E402
from lira_amd import _lib  # noqa: E402
from lira_amd.synthetic import CONFIGS, workload  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "sift1m"
data = sys.argv[2] if len(sys.argv) > 2 else "mixture"
opts = dict((a.split("=")[0], int(a.split("=")[1])) for a in sys.argv[3:])
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
dev = torch.device("cuda", 0)
x, c, assign, mk = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0, **opts).build(assign if assign.dim() == 2 else assign[:, None], x, B)
q = mk(nq, 1335)
probe = rank_nearest(q, c, nprobe)
lib = _lib.load()
lib.lira_debug_rs_clocks.argtypes = [ctypes.c_void_p]
v = (ctypes.c_uint64 * 16)()
for _ in range(3):
    idx.search(q, probe, k)
torch.cuda.synchronize()
lib.lira_debug_rs_clocks(v)
idx.set_profiling(True)
reps = 10
for _ in range(reps):
    idx.search(q, probe, k)
torch.cuda.synchronize()
pr = idx.profile_read()
lib.lira_debug_rs_clocks(v)
names = ["claim / between items", "item start", "done0 wait + barrier", "prologue (records, A operands)",
         "selection compares + queue", "thresholds + MFMAs + load waits", "drains (buffers, list merges)",
         "epilogue (merges, write-out)"]
tot = sum(v[i] for i in range(8))
waves = max(1, v[12])
print(f"{cfg}/{data}: scan {pr['scan_ms'] / max(1, pr['calls']):.3f} ms (clock build); {waves // reps} waves; "
      f"items/wave {v[9] / waves:.2f}, tiles/wave {v[10] / waves:.1f}, survivors/tile {v[11] / max(1, v[10]):.2f}, "
      f"row flushes/tile {v[13] / max(1, v[10]):.3f}")
for i, n in enumerate(names):
    print(f"  {n:36s} {v[i] / waves:12.0f} cycles/wave  {100.0 * v[i] / max(1, tot):5.1f} %")
