"""Repeat the clustered options case per screen variant; print mismatches vs the all-exact kernel."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lira-ann-search_amd"))
import numpy as np
import torch
from test_gpu_scan import clustered_case, make_index, run, bits

x, q, d2b, probe = clustered_case(61, 20000, 48, 8, 700, 3)
for order in (0, 1):
    idx = make_index(x, d2b, 8, "L2", order=order)
    for k in (10, 100):
        idx.set_option("screen", 0)
        De, Ie, _ = run(idx, q, probe, k)
        idx.set_option("screen", 1)
        for qr, ring in ((0, 0), (64, 2), (64, 4), (128, 3), (0, 0)):
            idx.set_option("qr", qr)
            idx.set_option("ring", ring)
            bad = []
            for rep in range(4):
                D, I, _ = run(idx, q, probe, k)
                bad.append(int((I != Ie).any(1).sum() + (bits(D) != bits(De)).any(1).sum()))
            print("order", order, "k", k, "qr", qr, "ring", ring, idx.describe(700, 3, k), "bad rows", bad, flush=True)
        idx.set_option("qr", 0)
        idx.set_option("ring", 0)
