"""Time lira_rank_nearest (and its GEMM alone) at a config's ranking shape, with
the probe lists checked against the oracle on a sample:
  python3 tools/rank_bench.py [nq B d nprobe]   (default: BIGANN-100M's 10000 1024 128 32)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lira-ann-search_amd"), os.path.join(ROOT, "oracle")]
import lira_amd  # noqa: E402
from lira_amd.index import RankWorkspace, centroid_gemm, rank_nearest  # noqa: E402

nq, B, d, nprobe = (int(a) for a in (sys.argv[1:5] if len(sys.argv) >= 5 else (10000, 1024, 128, 32)))
rng = np.random.default_rng(7)
c = (rng.random((B, d), dtype=np.float32) * 255).astype(np.float32)
q = (c[rng.integers(0, B, nq)] + 20 * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
dev = torch.device("cuda", 0)
qt, ct = torch.from_numpy(q).to(dev), torch.from_numpy(c).to(dev)
out = torch.empty((nq, nprobe), dtype=torch.int32, device=dev)
ws = RankWorkspace(nq, B, dev)


def timed(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


t_rank = timed(lambda: rank_nearest(qt, ct, nprobe, out=out, workspace=ws))
t_gemm = timed(lambda: centroid_gemm(qt, ct))
import oracle  # noqa: E402  (the checker, after the timed calls)
rows = np.r_[0:64, nq - 64:nq]
want = oracle.probe_nearest(oracle.centroid_dist(q[rows], c), nprobe)
same = bool(np.array_equal(out.cpu().numpy()[rows], want))
print(f"rank_nearest nq={nq} B={B} d={d} nprobe={nprobe}: {t_rank * 1e3:.1f} us per call "
      f"(centroid_gemm alone {t_gemm * 1e3:.1f} us); probe lists == oracle on {len(rows)} queries: {same}")
assert same
