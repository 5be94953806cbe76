"""GPU: the query-sharded path (lira_amd.distributed.sharded_search) and the
partition-sharded one (partition_sharded_search: per-rank bucket subsets,
all-gather, lira_merge_shards) over the real HIP index at world_size 2 -- both
ranks on cuda:0, gloo for the all-gather -- against the CPU oracle on the whole
batch; lira_merge_shards against the single full index."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, ROOT
from test_distributed import _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, nq, metric, out_dir):
    import sys
    for p in (PKG, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import oracle
    from lira_amd import PartitionedIndex, rank_nearest
    from lira_amd.distributed import sharded_search
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    rng = np.random.default_rng(5)
    n, d, b, k, nprobe = 30000, 40, 16, 10, 4
    c = rng.standard_normal((b, d), dtype=np.float32)
    x = (c[rng.integers(0, b, n)] + 0.5 * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    q = (c[rng.integers(0, b, nq)] + 0.5 * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
    d2b = rng.integers(0, b, (n, 2)).astype(np.int32)
    d2b[rng.random(n) < 0.7, 1] = -1
    dev = torch.device("cuda", 0)
    idx = PartitionedIndex.from_assignment(torch.from_numpy(x).to(dev), torch.from_numpy(d2b).to(dev), b, metric)
    ct = torch.from_numpy(c).to(dev)

    def search(qs, start):
        probe = rank_nearest(qs, ct, nprobe)
        D, I, _ = idx.search(qs, probe, k)
        return D, I

    D, I = sharded_search(search, torch.from_numpy(q).to(dev), gather_device="cpu")
    off, ids = oracle.build_csr(d2b, b)
    probe = oracle.probe_nearest(oracle.centroid_dist(q, c), nprobe)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Do, Io, _ = oracle.scan_topk(q, off, ids, x[ids], probe, k, met, idx.max_replicas)
    ok = np.array_equal(I.numpy(), Io) and np.array_equal(D.numpy().view(np.uint32), Do.view(np.uint32))
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("metric,nq", [("L2", 333), ("inner_product", 1000)])
def test_two_rank_sharded_hip_search(tmp_path, metric, nq):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, nq, metric, str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"r{r}").read() for r in range(2)] == ["ok", "ok"]


def _case(seed, n, d, b, nq, two=0.3):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((b, d), dtype=np.float32)
    x = (c[rng.integers(0, b, n)] + 0.5 * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    q = (c[rng.integers(0, b, nq)] + 0.5 * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
    d2b = rng.integers(0, b, (n, 2)).astype(np.int32)
    d2b[rng.random(n) >= two, 1] = -1
    return c, x, q, d2b


def _pworker(rank, world, port, metric, dedup, out_dir):
    import sys
    for p in (PKG, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import oracle
    from lira_amd import PartitionedIndex, rank_nearest
    from lira_amd.distributed import bucket_sizes, partition_owners, partition_sharded_search, shard_assignment
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    c, x, q, d2b = _case(8, 30000, 40, 16, 700)
    k, nprobe = 10, 5
    d2b_t = torch.from_numpy(d2b).to(dev)
    owners = partition_owners(bucket_sizes(d2b_t, 16), world)
    idx = PartitionedIndex(40, metric, 0).build(shard_assignment(d2b_t, owners, rank), torch.from_numpy(x).to(dev), 16)
    qt = torch.from_numpy(q).to(dev)
    probe = rank_nearest(qt, torch.from_numpy(c).to(dev), nprobe)
    D, I = partition_sharded_search(idx, qt, probe, k, dedup=dedup, gather_device="cpu")
    off, ids = oracle.build_csr(d2b, 16)
    probe_o = oracle.probe_nearest(oracle.centroid_dist(q, c), nprobe)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Do, Io, _ = oracle.scan_topk(q, off, ids, x[ids], probe_o, k, met, 2 if dedup else 0)
    ok = np.array_equal(I.cpu().numpy(), Io) and np.array_equal(D.cpu().numpy().view(np.uint32), Do.view(np.uint32))
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("metric,dedup", [("L2", True), ("inner_product", False)])
def test_two_rank_partition_shards_hip(tmp_path, metric, dedup):
    port = _free_port()
    mp.spawn(_pworker, args=(2, port, metric, dedup, str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"r{r}").read() for r in range(2)] == ["ok", "ok"]


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
@pytest.mark.parametrize("k", [1, 10, 100])
def test_merge_shards_equals_full_index(metric, k):
    # P virtual shards on one GPU: the merged per-shard results are the full
    # index's, bit for bit (replicas across shards: dedup on and off)
    import torch
    from lira_amd import PartitionedIndex, rank_nearest
    from lira_amd.distributed import bucket_sizes, merge_shards, partition_owners, shard_assignment
    dev = torch.device("cuda", 0)
    c, x, q, d2b = _case(21 + k, 20000, 24, 12, 300, two=0.5)
    xt, qt, d2b_t = (torch.from_numpy(a).to(dev) for a in (x, q, d2b))
    full = PartitionedIndex(24, metric, 0).build(d2b_t, xt, 12)
    probe = rank_nearest(qt, torch.from_numpy(c).to(dev), 6)
    probe[::5, 4:] = -1
    for dedup in (True, False):
        Df, If, _ = full.search(qt, probe, k, dedup=dedup)
        for P in (1, 2, 3, 8):
            own = partition_owners(bucket_sizes(d2b_t, 12), P)
            parts = []
            for r in range(P):
                sh = PartitionedIndex(24, metric, 0).build(shard_assignment(d2b_t, own, r), xt, 12)
                parts.append(sh.search(qt, probe, k, dedup=dedup)[:2])
                del sh
            Dm, Im = merge_shards(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]),
                                  metric, dedup)
            assert torch.equal(Im, If), (P, dedup)
            assert torch.equal(Dm.view(torch.int32), Df.view(torch.int32)), (P, dedup)


def test_merge_shards_pads_and_empty():
    import torch
    from lira_amd import LiraError
    from lira_amd.distributed import merge_shards
    dev = torch.device("cuda", 0)
    inf = float("inf")
    # shard 0: two results, shard 1: one equal to shard 0's first (a replica), shard 2: nothing
    D = torch.tensor([[[1.0, 2.0, inf, inf]], [[1.0, 3.0, inf, inf]], [[inf] * 4]], device=dev)
    I = torch.tensor([[[5, 7, -1, -1]], [[5, 9, -1, -1]], [[-1] * 4]], device=dev)
    Dm, Im = merge_shards(D, I, "L2", True)
    assert Im.tolist() == [[5, 7, 9, -1]] and Dm.tolist() == [[1.0, 2.0, 3.0, inf]]
    Dm, Im = merge_shards(D, I, "L2", False)
    assert Im.tolist() == [[5, 5, 7, 9]]
    # IP: descending inner products, ties -> smaller id
    Dip = torch.tensor([[[4.0, 2.0]], [[4.0, 3.0]]], device=dev)
    Iip = torch.tensor([[[8, 1]], [[6, 2]]], device=dev)
    Dm, Im = merge_shards(Dip, Iip, "inner_product", True)
    assert Im.tolist() == [[6, 8]] and Dm.tolist() == [[4.0, 4.0]]
    e = merge_shards(torch.empty((2, 0, 3), device=dev), torch.empty((2, 0, 3), dtype=torch.int64, device=dev))
    assert e[0].shape == (0, 3)
    with pytest.raises(LiraError):
        merge_shards(torch.empty((65, 1, 3), device=dev), torch.empty((65, 1, 3), dtype=torch.int64, device=dev))
