"""the PER_PARTITION route on a centred IP index (DEEP10M-shaped lists)
falls back from k_screen_r to the fp32-tile screens.  Time it next to the default route on
the same index and batch: python3 tools/pp_ip_bench.py [n d B nq nprobe k]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lira-ann-search_amd"))
import lira_amd  # noqa: E402

n, d, B, nq, nprobe, k = (int(a) for a in (sys.argv[1:7] if len(sys.argv) >= 7 else (2000000, 96, 256, 2000, 32, 100)))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
c = torch.nn.functional.normalize(torch.randn(B, d, device=dev, generator=g), dim=1)
lab = torch.randint(0, B, (n,), device=dev, generator=g)
x = torch.nn.functional.normalize(c[lab] + 0.35 * torch.randn(n, d, device=dev, generator=g), dim=1)
q = torch.nn.functional.normalize(c[torch.randint(0, B, (nq,), device=dev, generator=g)]
                                  + 0.35 * torch.randn(nq, d, device=dev, generator=g), dim=1)
idx = lira_amd.PartitionedIndex.from_assignment(x, lab.to(torch.int32)[:, None], B, "inner_product", 0)
probe = lira_amd.rank_nearest(q, c, nprobe)


def timed(**kw):
    idx.search(q, probe, k, **kw)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        idx.search(q, probe, k, **kw)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 5


t_def = timed()
t_pp = timed(per_partition=True)
print(f"IP n={n} d={d} B={B} nq={nq} nprobe={nprobe} k={k}: default {t_def:.2f} ms "
      f"[{idx.describe(nq, nprobe, k)[:60]}], PER_PARTITION {t_pp:.2f} ms")
