"""Stress one wide-screen case and describe every mismatch against the oracle (GPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lira-ann-search_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from test_gpu_scan import bits, make_index, random_case, run  # noqa: E402

d = int(sys.argv[1]) if len(sys.argv) > 1 else 33
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
x, q, d2b, probe = random_case(200 + d, 3000, d, 6, 33, 3, "L2")
off, ids = oracle.build_csr(d2b, 6)
vecs = oracle.gather_lists(x, off, ids)
Do, Io, nco = oracle.scan_topk(q, off, ids, vecs, probe, 10, oracle.L2, 1)
nbad = 0
for it in range(reps):
    if it % 10 == 0:
        idx = make_index(x, d2b, 6, "L2")
    D, I, nc = run(idx, q, probe, 10)
    rows = np.where((I != Io).any(1) | (bits(D) != bits(Do)).any(1))[0]
    if len(rows):
        nbad += 1
        r = rows[0]
        miss = [int(v) for v in Io[r] if v not in I[r]]
        where = [int(b) for v in miss for b in range(6) if v in ids[off[b]:off[b + 1]]]
        print(f"rep {it}: {len(rows)} rows bad, row {r} probe {probe[r]} missing {miss} in lists {where}\n"
              f"  gpu {I[r]} {D[r]}\n  ora {Io[r]} {Do[r]}", flush=True)
print("bad reps", nbad, "of", reps, flush=True)
