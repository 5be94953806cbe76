"""CPU: the query-sharded path (lira_amd.distributed) at world_size 2 over gloo.

Each rank searches its slice with the CPU oracle (standing in for the GPU
scan, which the -m gpu tests cover) and the all-gather must reproduce the
single-process result bit for bit, including uneven slices.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nq, out_dir):
    import sys
    for p in (PKG, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle
    from lira_amd.distributed import sharded_search
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((3000, 16), dtype=np.float32)
    d2b = rng.integers(0, 6, (3000, 1)).astype(np.int32)
    off, ids = oracle.build_csr(d2b, 6)
    vecs = x[ids]
    q = torch.from_numpy(rng.standard_normal((nq, 16), dtype=np.float32))
    probe = rng.integers(0, 6, (nq, 3)).astype(np.int32)

    def search(qs, s):
        D, I, _ = oracle.scan_topk(qs.numpy(), off, ids, vecs, probe[s:s + qs.shape[0]], 7)
        return torch.from_numpy(D), torch.from_numpy(I)

    D, I = sharded_search(search, q)
    Dw, Iw, _ = oracle.scan_topk(q.numpy(), off, ids, vecs, probe, 7)
    ok = np.array_equal(I.numpy(), Iw) and np.array_equal(D.numpy().view(np.uint32), Dw.view(np.uint32))
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("nq", [10, 11])
def test_two_rank_gloo_sharded_search(tmp_path, nq):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, nq, str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"r{r}").read() for r in range(2)] == ["ok", "ok"]


def test_shard_bounds_cover_exactly():
    from lira_amd.distributed import shard_bounds
    for n in (0, 1, 7, 10000, 10001):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
