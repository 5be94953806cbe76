"""CPU: the query-sharded and partition-sharded paths (lira_amd.distributed) at
world_size 2 over gloo.

Each rank searches with the CPU oracle (standing in for the GPU scan, which the
-m gpu tests cover) and the exchange must reproduce the single-process result
bit for bit: the all-gather of query slices (uneven slices included), and for
partition shards the all-gather of every rank's top-k over its own buckets plus
the k-way merge (oracle.merge_shards, the restatement of lira_merge_shards, whose
device form is checked against the full index in tests/test_gpu_distributed.py).
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


def _pworker(rank, world, port, metric, dedup, out_dir):
    import sys
    for p in (PKG, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle
    from lira_amd.distributed import bucket_sizes, gather_shards, partition_owners, shard_assignment
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(3)
    n, d, b, k, nq = 4000, 16, 9, 12, 40
    x = rng.standard_normal((n, d), dtype=np.float32)
    # two buckets per row for 40 % of the rows: replicas that land on both ranks
    d2b = rng.integers(0, b, (n, 2)).astype(np.int32)
    d2b[rng.random(n) < 0.6, 1] = -1
    q = rng.standard_normal((nq, d), dtype=np.float32)
    probe = np.stack([rng.permutation(b)[:5] for _ in range(nq)]).astype(np.int32)
    probe[::7, 3:] = -1
    met = oracle.IP if metric == "inner_product" else oracle.L2
    owners = partition_owners(bucket_sizes(torch.from_numpy(d2b), b), world)
    mine = shard_assignment(torch.from_numpy(d2b), owners, rank).numpy()
    off, ids = oracle.build_csr(mine, b)
    D, I, _ = oracle.scan_topk(q, off, ids, x[ids], probe, k, met, 2 if dedup else 0)
    Dp, Ip = gather_shards(torch.from_numpy(D), torch.from_numpy(I), world)
    Dm, Im = oracle.merge_shards(Dp.numpy(), Ip.numpy(), metric == "inner_product", dedup, k)
    off, ids = oracle.build_csr(d2b, b)
    Dw, Iw, _ = oracle.scan_topk(q, off, ids, x[ids], probe, k, met, 2 if dedup else 0)
    ok = np.array_equal(Im, Iw) and np.array_equal(Dm.view(np.uint32), Dw.view(np.uint32))
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("metric,dedup", [("L2", True), ("L2", False), ("inner_product", True)])
def test_two_rank_gloo_partition_shards(tmp_path, metric, dedup):
    port = _free_port()
    mp.spawn(_pworker, args=(2, port, metric, dedup, str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"r{r}").read() for r in range(2)] == ["ok", "ok"]


def test_partition_owners_balance_and_masking():
    from lira_amd.distributed import bucket_sizes, partition_owners, shard_assignment
    rng = np.random.default_rng(9)
    sizes = rng.integers(0, 5000, 1024)
    for w in (1, 2, 3, 8):
        own = partition_owners(sizes, w)
        assert np.array_equal(own, partition_owners(sizes, w))  # deterministic
        assert set(np.unique(own)) <= set(range(w))
        load = np.bincount(own, weights=sizes, minlength=w)
        assert load.max() - load.min() <= sizes.max()  # greedy LPT bound
    d2b = torch.from_numpy(rng.integers(-1, 12, (500, 2)).astype(np.int32))
    s = bucket_sizes(d2b, 12)
    assert s.sum() == int((d2b >= 0).sum())
    own = partition_owners(s, 3)
    parts = [shard_assignment(d2b, own, r) for r in range(3)]
    # every valid slot kept by exactly its owner, nothing else kept
    kept = sum((p >= 0).to(torch.int64) for p in parts)
    assert torch.equal(kept, (d2b >= 0).to(torch.int64))
    for r, p in enumerate(parts):
        v = p[p >= 0].numpy()
        assert np.all(own[v] == r)
