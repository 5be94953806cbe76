"""Repeat golden / random wide-screen cases and count mismatching runs (GPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lira-ann-search_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from test_gpu_scan import bits, make_index, run  # noqa: E402
from conftest import load_golden  # noqa: E402

g = load_golden("sift_like_redundant")
k = int(g["k"])
for fresh in range(3):
    idx = make_index(g["x"], g["data_2_bkt"], g["centroids"].shape[0], str(g["metric"]))
    for share in (1, 0):
        idx.set_option("share", share)
        bad = []
        for rep in range(20):
            D, I, nc = run(idx, g["q"], g["probe"], k)
            rows = np.where((I != g["I"]).any(1) | (bits(D) != bits(g["D"])).any(1))[0]
            if len(rows):
                bad.append((rep, rows.tolist()[:5]))
        print("index", fresh, "share", share, "bad runs", len(bad), bad[:3], flush=True)
    if fresh == 0 and bad:
        r = bad[0][1][0]
        print("row", r, "probe", g["probe"][r], "\n gpu", I[r], D[r], "\n want", g["I"][r], g["D"][r])
