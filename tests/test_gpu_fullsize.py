"""GPU: BASELINE.json shapes end to end (rank -> scan -> top-k) with the oracle
on a query sample and size-independent properties on the whole batch."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def build(cfg, nq, seed=1234, n_override=None, data="mixture"):
    from lira_amd import PartitionedIndex
    from lira_amd.synthetic import CONFIGS, workload
    N, d, B, nprobe, k, metric, _ = CONFIGS[cfg]
    N = n_override or N
    dev = torch.device("cuda", 0)
    x, c, assign, make_queries = workload(cfg, seed, dev, data, n_override=N)
    idx = PartitionedIndex(d, metric, 0).build(assign[:, None], x, B)
    off = np.zeros(B + 1, dtype=np.int64)
    off[1:] = np.cumsum(idx.list_sizes)
    ids = torch.from_numpy(np.concatenate([idx.list_ids(b) for b in range(B)]))
    q = make_queries(nq, seed + 1)
    return idx, x, c, q, off, ids, (N, d, B, nprobe, k, metric)


# mixture: separated clusters, the pruning skips most blocks; latent: k-means
# cells over a continuum, the pruning rarely fires (lira_amd/synthetic.py)
@pytest.mark.parametrize("cfg,nq,n,data", [("sift1m", 10000, None, "mixture"), ("gist1m", 1000, 200_000, "mixture"),
                                           ("deep10m", 2000, 1_000_000, "mixture"),
                                           ("sift1m", 10000, None, "latent"), ("gist1m", 1000, 200_000, "latent"),
                                           ("deep10m", 2000, 1_000_000, "latent")])
def test_fullsize(cfg, nq, n, data):
    from lira_amd import rank_nearest
    idx, x, c, q, off, ids, (N, d, B, nprobe, k, metric) = build(cfg, nq, n_override=n, data=data)
    probe = rank_nearest(q, c, nprobe)
    D, I, nc = idx.search(q, probe, k)
    torch.cuda.synchronize()
    idx.check()
    Dn, In, ncn = D.cpu().numpy(), I.cpu().numpy(), nc.cpu().numpy()
    # properties over the whole batch
    assert (In >= 0).all() and (In < N).all()
    if metric == "L2":
        assert (np.diff(Dn, axis=1) >= 0).all()
    else:
        assert (np.diff(Dn, axis=1) <= 0).all()
    assert all(len(set(r)) == k for r in In[:500])  # dedup: unique ids
    sizes = np.diff(off)
    pr = probe.cpu().numpy()
    assert np.array_equal(ncn, sizes[pr].sum(1))
    # oracle parity on a sample (bit-exact ids and distances)
    s = np.r_[0:32, nq - 32:nq]
    xs, ids_np = x.cpu().numpy(), ids.cpu().numpy()
    met = oracle.IP if metric == "inner_product" else oracle.L2
    qs = q.cpu().numpy()[s]
    assert np.array_equal(pr[s], oracle.probe_nearest(oracle.centroid_dist(qs, c.cpu().numpy()), nprobe))
    Do, Io, _ = oracle.scan_topk(qs, off, ids_np, xs[ids_np], pr[s], k, met, 1)
    assert np.array_equal(In[s], Io)
    assert np.array_equal(Dn[s].view(np.uint32), Do.view(np.uint32))
    # the same batch again gives the same bits (determinism)
    D2, I2, _ = idx.search(q, probe, k)
    assert torch.equal(I2, I) and torch.equal(D2.view(torch.int32), D.view(torch.int32))
