"""Diagnostic: the plan's group-0 chunk size (head[19]) and the seed's work
estimate (head[64..127]) for one scan of a config (caller-owned workspace).
usage: python tools/plan_dbg.py <config> <data>"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lira-ann-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lira_amd import PartitionedIndex, rank_nearest, _lib  # noqa: E402
from lira_amd.synthetic import CONFIGS, workload  # noqa: E402

cfg, data = sys.argv[1], sys.argv[2]
N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
dev = torch.device("cuda", 0)
x, c, assign, mq = workload(cfg, 1234, dev, data)
idx = PartitionedIndex(d, metric, 0).build(assign[:, None] if assign.dim() == 1 else assign, x, B)
q = mq(nq, 1335)
probe = rank_nearest(q, c, nprobe)
sz = ctypes.c_size_t()
_lib.call("lira_scan_workspace_size", idx.handle, nq, nprobe, k, 0, ctypes.byref(sz))
ws = torch.zeros(sz.value, dtype=torch.uint8, device=dev)
D = torch.empty((nq, k), dtype=torch.float32, device=dev)
I = torch.empty((nq, k), dtype=torch.int64, device=dev)
nc = torch.empty(nq, dtype=torch.int64, device=dev)
_lib.call("lira_scan_topk", idx.handle, _lib.ptr(q), nq, _lib.ptr(probe), nprobe, k, 0,
          _lib.ptr(D), _lib.ptr(I), _lib.ptr(nc), _lib.ptr(ws), sz.value, _lib.stream_ptr())
torch.cuda.synchronize()
r256 = lambda b: (b + 255) & ~255  # noqa: E731
off_head = 2 * r256(2 * B * 4)
h = ws[off_head:off_head + 512].cpu().numpy().view(np.int32)
print(cfg, data, "describe", idx.describe(nq, nprobe, k))
print("head[19] (group-0 chunk blocks)", h[19], "work estimate sum", int(h[64:128].astype(np.int64).sum()),
      "items", h[1], "queues", h[10:19])
