"""Run one golden case step by step (GPU), printing after each synchronised step."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lira-ann-search_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from test_gpu_scan import bits, make_index, run  # noqa: E402
from conftest import load_golden  # noqa: E402

name = sys.argv[1]
wide = int(sys.argv[2])
g = load_golden(name)
k = int(g["k"])
idx = make_index(g["x"], g["data_2_bkt"], g["centroids"].shape[0], str(g["metric"]))
idx.set_option("wide", wide)
print("built", idx.describe(g["q"].shape[0], g["probe"].shape[1], k), flush=True)
for kw in ({}, {"dedup": False}):
    t = time.time()
    D, I, nc = run(idx, g["q"], g["probe"], k, **kw)
    print(kw, "ok" if np.array_equal(I, g["I" if not kw else "I_nodedup"]) else "DIFF", time.time() - t, flush=True)
