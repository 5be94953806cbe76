"""GPU: the query-sharded path (lira_amd.distributed.sharded_search) over the
real HIP index at world_size 2 -- both ranks on cuda:0, gloo for the
all-gather -- against the CPU oracle on the whole batch."""
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
