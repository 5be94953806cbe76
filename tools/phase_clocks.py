"""Per-phase cycle split of the screen kernel (LIRA_OPT_DEBUG bit 8: thread 0 of
every workgroup adds clock64() deltas: item prologue -> stats[1], block loop ->
stats[3], epilogue -> stats[6]).  Timing experiment only (debug bits 1/2/4 also
switch off MFMA / selection / staging; results invalid).  Needs a debug build
(production libraries refuse LIRA_OPT_DEBUG != 0):
  VARIANT_FLAGS=-DLIRA_PHASE_CLOCKS tools/build_variant.sh lira_screen.hip \
      lira-ann-search_amd/csrc/lira_screen.hip clk && LIRA_HIP_LIB=variants/clk.so python tools/phase_clocks.py ...

usage: python tools/phase_clocks.py <config> <data> <debug bits> [option=value ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lira-ann-search_amd"))
import torch  # noqa: E402

from lira_amd import PartitionedIndex, rank_nearest  # noqa: E402
from lira_amd.synthetic import CONFIGS, workload  # noqa: E402

cfg, data, dbg = sys.argv[1], sys.argv[2], int(sys.argv[3])
opts = dict((a.split("=")[0], int(a.split("=")[1])) for a in sys.argv[4:])
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
nq = int(os.environ.get("NQ", nq))  # (NQ=1250: the 8-GPU strong-scaling share)
dev = torch.device("cuda", 0)
x, c, assign, mq = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0, **opts).build(assign[:, None] if assign.dim() == 1 else assign, x, B)
q = mq(nq, 1335)
probe = rank_nearest(q, c, nprobe)
for _ in range(3):
    idx.search(q, probe, k)
idx.set_stats(True)
idx.search(q, probe, k)
work = idx.stats_read()  # (the work counters are off while the clocks run)
idx.set_option("debug", dbg | 8 | opts.get("debug", 0))
idx.set_profiling(True)
idx.search(q, probe, k)
torch.cuda.synchronize()
st = idx.stats_read()
pr = idx.profile_read()
print(cfg, data, "debug", dbg, opts, "kernel", idx.describe(nq, nprobe, k))
tot = max(1, st["chunks_nominal"] + st["blocks_dropped"] + st["rescans"])
print("scan_ms %.3f  cycles: prologue %.3g  blocks %.3g  epilogue %.3g  (fractions %.2f / %.2f / %.2f)" % (
    pr["scan_ms"], st["chunks_nominal"], st["blocks_dropped"], st["rescans"],
    st["chunks_nominal"] / tot, st["blocks_dropped"] / tot, st["rescans"] / tot))
# k_screen_m: wave 0's block loop split (refresh + skip test / chunk loop / selection)
bl = max(1, st["blocks_dropped"])
print("block loop: refresh %.2f  chunks %.2f  selection %.2f  (slow-path regs %d)  per block: %.0f / %.0f / %.0f cycles"
      % (st["chunks_computed"] / bl, st["blocks"] / bl, st["blocks_skipped"] / bl, st["survivors"],
         st["chunks_computed"] / max(1, work["blocks"]), st["blocks"] / max(1, work["blocks"]),
         st["blocks_skipped"] / max(1, work["blocks"])))
print("chunk-start waits + barriers: %.0f cycles per block (%.2f of the chunk loop)" % (
    st["rechecked"] / max(1, work["blocks"]), st["rechecked"] / max(1, st["blocks"])))
print("blocks", work["blocks"], "skipped", work["blocks_skipped"], "survivors", work["survivors"])
