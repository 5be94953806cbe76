"""Diagnostic: run one scan of a bench config with a caller-owned workspace and
print the event counters a STATS build of lira_scan.hip leaves in head[2..8]
(in-loop flushes, final flushes, rows-with-survivors, blocks, items, bound
computations, survivor-lanes).  LIRA_HIP_LIB must point at that build.
usage: python tools/scan_stats.py [config]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lira-ann-search_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(cfg="sift1m"):
    from lira_amd import PartitionedIndex, rank_nearest, _lib
    from lira_amd.synthetic import CONFIGS, mixture_torch, nearest_centre
    N, d, B, nprobe, k, metric, nq = CONFIGS[cfg]
    dev = torch.device("cuda", 0)
    x, c = mixture_torch(N, d, B, 1234, dev)
    idx = PartitionedIndex(d, metric, 0).build(nearest_centre(x, c)[:, None], x, B)
    q, _ = mixture_torch(nq, d, B, 1235, dev, centres=c)
    probe = rank_nearest(q, c, nprobe)
    sz = ctypes.c_size_t()
    _lib.call("lira_scan_workspace_size", idx.handle, nq, nprobe, k, 1, ctypes.byref(sz))
    ws = torch.zeros(sz.value, dtype=torch.uint8, device=dev)
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    nc = torch.empty(nq, dtype=torch.int64, device=dev)
    _lib.call("lira_scan_topk", idx.handle, _lib.ptr(q), nq, _lib.ptr(probe), nprobe, k, 1,
              _lib.ptr(D), _lib.ptr(I), _lib.ptr(nc), _lib.ptr(ws), sz.value, _lib.stream_ptr())
    torch.cuda.synchronize()
    r256 = lambda b: (b + 255) & ~255  # noqa: E731
    off_head = 2 * r256(B * 4)
    h = ws[off_head:off_head + 64].cpu().numpy().view(np.int32)
    names = ["next", "n_items", "flush_loop", "flush_final", "rows_with_surv", "blocks(wave)",
             "items", "bound_calc", "surv_lanes"]
    print(cfg, os.environ.get("LIRA_SCAN_TWO_PHASE", "1"), {n: int(v) for n, v in zip(names, h[:9])})


if __name__ == "__main__":
    main(*sys.argv[1:2])
