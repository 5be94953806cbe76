"""GPU: every BASELINE.json config at its real shape end to end (rank -> scan ->
top-k), with the oracle on a query sample and size-independent properties on
the whole batch (search.cpp:413-548; BIGANN-100M on LIRA_largescale.py's full
redundancy, n_mul = 2, LIRA_largescale.py:37-39)."""
import gc

import numpy as np
import pytest
import torch

import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def build(cfg, nq, seed=1234, data="mixture", **options):
    from lira_amd import PartitionedIndex
    from lira_amd.synthetic import CONFIGS, workload
    N, d, B, nprobe, k, metric, _ = CONFIGS[cfg]
    dev = torch.device("cuda", 0)
    x, c, assign, make_queries = workload(cfg, seed, dev, data)
    idx = PartitionedIndex(d, metric, 0, **options).build(assign if assign.dim() == 2 else assign[:, None], x, B)
    del assign
    q = make_queries(nq, seed + 1)
    return idx, x, c, q, (N, d, B, nprobe, k, metric)


def properties(idx, q, probe, D, I, nc, N, k, metric):
    """Size-independent checks over the whole batch."""
    Dn, In, ncn = D.cpu().numpy(), I.cpu().numpy(), nc.cpu().numpy()
    assert (In >= 0).all() and (In < N).all()
    if metric == "L2":
        assert (np.diff(Dn, axis=1) >= 0).all()
    else:
        assert (np.diff(Dn, axis=1) <= 0).all()
    srt = np.sort(In, axis=1)
    assert (np.diff(srt, axis=1) > 0).all()  # dedup: k distinct ids per query
    sizes = np.asarray(idx.list_sizes)
    assert np.array_equal(ncn, sizes[probe.cpu().numpy()].sum(1))
    return Dn, In


def oracle_sample(idx, x, q, probe, rows, k, metric, lists=None):
    """search.cpp's scan over each sampled query's own probed lists (a per-query
    sub-CSR, so an index larger than host memory can be checked)."""
    met = oracle.IP if metric == "inner_product" else oracle.L2
    cache = {}

    def list_ids(b):
        if lists is not None:
            return lists[b]
        if b not in cache:
            cache[b] = idx.list_ids(b)
        return cache[b]

    def gather(ids):
        return x[torch.from_numpy(ids).to(x.device).long()].cpu().numpy()

    return oracle.scan_topk_sampled(q.cpu().numpy()[rows], probe.cpu().numpy()[rows], list_ids, gather, k, met,
                                    idx.max_replicas)


# mixture: separated clusters, the pruning skips most blocks; latent: k-means
# cells over a continuum, the pruning rarely fires (lira_amd/synthetic.py)
@pytest.mark.parametrize("cfg,nq,data", [("sift1m", 10000, "mixture"), ("sift1m", 10000, "latent"),
                                         ("gist1m", 1000, "mixture"), ("gist1m", 1000, "latent"),
                                         ("deep10m", 10000, "mixture"), ("deep10m", 10000, "latent")])
def test_fullsize(cfg, nq, data):
    from lira_amd import rank_nearest
    gc.collect()
    torch.cuda.empty_cache()
    idx, x, c, q, (N, d, B, nprobe, k, metric) = build(cfg, nq, data=data)
    assert idx.ntotal == N
    probe = rank_nearest(q, c, nprobe)
    D, I, nc = idx.search(q, probe, k)
    torch.cuda.synchronize()
    idx.check()
    Dn, In = properties(idx, q, probe, D, I, nc, N, k, metric)
    # oracle parity on a sample (bit-exact ids and distances); probe lists too
    s = np.r_[0:32, nq - 32:nq]
    pr = probe.cpu().numpy()
    assert np.array_equal(pr[s], oracle.probe_nearest(oracle.centroid_dist(q.cpu().numpy()[s], c.cpu().numpy()),
                                                      nprobe))
    lists = [idx.list_ids(b) for b in range(B)]
    Do, Io = oracle_sample(idx, x, q, probe, s, k, metric, lists)
    assert np.array_equal(In[s], Io)
    assert np.array_equal(Dn[s].view(np.uint32), Do.view(np.uint32))
    # the same batch again gives the same bits (determinism)
    D2, I2, _ = idx.search(q, probe, k)
    assert torch.equal(I2, I) and torch.equal(D2.view(torch.int32), D.view(torch.int32))
    del idx, x


@pytest.mark.timeout(900)
def test_bigann100m_full_redundancy():
    """BIGANN-100M shape on the LIRA_largescale.py path: every row in its 2
    nearest partitions (2e8 stored rows), the compact index (row-major +
    split-bf16 copies, no fp32 tiles) so it fits one MI355X's HBM."""
    from lira_amd import rank_nearest
    gc.collect()
    torch.cuda.empty_cache()
    idx, x, c, q, (N, d, B, nprobe, k, metric) = build("bigann100m", 10000, keep_tiles=False)
    assert idx.ntotal == 2 * N and idx.max_replicas == 2 and not idx.has_tiles
    assert idx.memory_bytes() <= 250e9
    probe = rank_nearest(q, c, nprobe)
    D, I, nc = idx.search(q, probe, k)
    torch.cuda.synchronize()
    idx.check()
    Dn, In = properties(idx, q, probe, D, I, nc, N, k, metric)
    rows = np.r_[0:32, 10000 - 32:10000]
    Do, Io = oracle_sample(idx, x, q, probe, rows, k, metric)
    assert np.array_equal(In[rows], Io)
    assert np.array_equal(Dn[rows].view(np.uint32), Do.view(np.uint32))
    del idx, x
