import sys, os
sys.path.insert(0, "lira-ann-search_amd"); sys.path.insert(0, "oracle")
import numpy as np, torch
import oracle
from lira_amd import rank_nearest
for (nq, nb, d) in [(4100, 256, 96), (257, 130, 96), (4097, 200, 64)]:
    rng = np.random.default_rng(nq * 7 + nb)
    c = rng.standard_normal((nb, d), dtype=np.float32)
    q = (c[rng.integers(0, nb, nq)] + 0.3 * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
    qt, ct = torch.from_numpy(q).cuda(), torch.from_numpy(c).cuda()
    cd = oracle.centroid_dist(q, c)
    for nprobe in [64, 256 if nb >= 256 else nb]:
        got = rank_nearest(qt, ct, nprobe).cpu().numpy()
        want = oracle.probe_nearest(cd, nprobe)
        bad = np.argwhere(got != want)
        print(nq, nb, d, nprobe, "mismatches", len(bad), "rows", len(set(bad[:, 0])) if len(bad) else 0)
        for r, p in bad[:5]:
            print("  row", r, "pos", p, "got", got[r, p], "want", want[r, p], "d_got", cd[r, got[r, p]] if got[r,p] >= 0 else None, "d_want", cd[r, want[r, p]])
