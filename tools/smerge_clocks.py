"""Phase split of k_smerge (timing experiment; needs the clock variant library:
tools/build_variant.sh lira_screen.hip <source with g_sm_clk stamps> smclk).
usage: LIRA_HIP_LIB=variants/smclk.so python tools/smerge_clocks.py [config] [data]"""
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
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
dev = torch.device("cuda", 0)
x, c, assign, mk = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0).build(assign if assign.dim() == 2 else assign[:, None], x, B)
q = mk(nq, 1335)
probe = rank_nearest(q, c, nprobe)
lib = _lib.load()
lib.lira_debug_smerge_clocks.argtypes = [ctypes.c_void_p]
v = (ctypes.c_uint64 * 8)()
for _ in range(3):
    idx.search(q, probe, k)
torch.cuda.synchronize()
lib.lira_debug_smerge_clocks(v)
reps = 10
for _ in range(reps):
    idx.search(q, probe, k)
torch.cuda.synchronize()
lib.lira_debug_smerge_clocks(v)
names = ["prologue (bound, candidate count)", "take_lists (list walk)", "spill records",
         "last exact re-check + merge", "emit"]
tot = sum(v[i] for i in range(5))
waves = max(1, v[5])
print(f"{cfg}/{data}: {waves // reps} query waves per call, rechecked {v[6] / waves:.1f} per query")
for i, n in enumerate(names):
    print(f"  {n:32s} {v[i] / waves:10.0f} cycles/wave  {100.0 * v[i] / max(1, tot):5.1f} %")
