"""Diagnose k_screen_w mismatches against the oracle on one test case (GPU)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lira-ann-search_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from test_gpu_scan import bits, make_index, random_case, run  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 48
n, b, nq, nprobe, k = 60000, 10, 1500, 4, 10
x, q, d2b, probe = random_case(300 + d, n, d, b, nq, nprobe, "L2")
idx = make_index(x, d2b, b, "L2")
print(idx.describe(nq, nprobe, k))
off, ids = oracle.build_csr(d2b, b)
vecs = oracle.gather_lists(x, off, ids)
Do, Io, nco = oracle.scan_topk(q, off, ids, vecs, probe, k, oracle.L2, idx.max_replicas)
for opts in ({}, {"wide": 0}, {"prune": 0}, {"seed": 0}, {"rounds": 64}, {"share": 0}):
    for kk, v in opts.items():
        idx.set_option(kk, v)
    idx.set_stats(True)
    D, I, nc = run(idx, q, probe, k)
    st = idx.stats_read()
    idx.set_stats(False)
    bad = np.where((I != Io).any(1) | (bits(D) != bits(Do)).any(1))[0]
    print(opts, "bad rows", len(bad), "stats", st)
    for r in bad[:3]:
        print("  row", r, "probe", probe[r], "\n   gpu", I[r], D[r], "\n   ora", Io[r], Do[r])
    for kk in opts:
        idx.set_option(kk, {"wide": 1, "prune": 1, "seed": 1, "rounds": 0, "share": 1}[kk])
