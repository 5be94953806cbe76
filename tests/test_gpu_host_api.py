"""GPU: LIRA's query-path helpers (lira_amd.utils) and the search.cpp engine
(lira_amd.search) against the oracle and plain-Python restatements."""
import types

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def mixture(n, d, b, seed):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((b, d), dtype=np.float32)
    x = (c[rng.integers(0, b, n)] + 0.35 * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    return x, c, rng


def test_get_dist_cid():
    from scipy.spatial.distance import cdist

    from lira_amd.utils import get_dist_cid
    x, c, _ = mixture(3000, 24, 10, 0)
    km = types.SimpleNamespace(centroids=c)
    got = get_dist_cid(x, km, 10)
    assert np.array_equal(got.view(np.uint32), oracle.centroid_dist(x, c).view(np.uint32))
    assert np.allclose(got, cdist(x, c).astype(np.float32), rtol=1e-5)  # utils.py:115


def test_get_cmp_recall_and_bucket_views():
    from lira_amd.utils import create_inner_indexes, get_cmp_recall
    x, c, rng = mixture(5000, 32, 12, 1)
    lab = oracle.centroid_dist(x, c).argmin(1)
    # insertion order, with a few redundant ids appended (LIRA_smallscale.py:94-97)
    cluster_ids = [list(np.where(lab == b)[0]) for b in range(12)]
    for t in rng.choice(5000, 50, replace=False):
        cluster_ids[(lab[t] + 1) % 12].append(int(t))
    cluster_ids[11] = cluster_ids[11][:4]  # a bucket with fewer than k rows
    cfg = types.SimpleNamespace(k=10, n_bkt=12, dis_metric="L2")
    q = (c[rng.integers(0, 12, 60)] + 0.35 * rng.standard_normal((60, 32), dtype=np.float32)).astype(np.float32)
    inner = create_inner_indexes(x, cluster_ids, cfg)
    assert [v.ntotal for v in inner] == [len(b) for b in cluster_ids]
    t, cmp_, found = get_cmp_recall(inner, q, cluster_ids, cfg)
    assert t.shape == (60, 12) and (cmp_ == np.array([len(b) for b in cluster_ids])).all()
    # measured per bucket (one timed launch each), the same for every query of the batch
    assert (t > 0).all() and np.allclose(t, t[:1]) and (t < 1.0).all()
    t2, _, found2 = get_cmp_recall(inner, q, cluster_ids, cfg, timing="apportion")
    assert np.array_equal(found2, found) and (t2 > 0).all()
    with pytest.raises(ValueError):
        get_cmp_recall(inner, q, cluster_ids, cfg, timing="per-query")
    off = np.zeros(13, np.int64)
    off[1:] = np.cumsum([len(b) for b in cluster_ids])
    ids = np.concatenate([np.asarray(b, np.int32) for b in cluster_ids])
    probe = np.tile(np.arange(12, dtype=np.int32), (60, 1))
    _, Io = oracle.scan_per_partition(q, off, ids, x[ids], probe, 10)
    assert np.array_equal(found, Io)
    assert (found[:, 11, 4:] == -1).all()
    # faiss-like per-bucket search returns positions in the bucket's insertion order
    D, pos = inner[3].search(q[:5], 10)
    assert np.array_equal(np.asarray(cluster_ids[3])[pos], found[:5, 3])


def test_query_tuning_matches_python_restatement():
    from lira_amd.utils import get_knn_distr_redundancy, query_tuning
    rng = np.random.default_rng(2)
    nq, nb, k = 40, 8, 5
    d2b = np.full((300, 2), -1, np.int64)
    d2b[:, 0] = rng.integers(0, nb, 300)
    d2b[:30, 1] = rng.integers(0, nb, 30)
    gt = np.stack([rng.choice(300, k, replace=False) for _ in range(nq)])
    cfg = types.SimpleNamespace(k=k, n_bkt=nb)
    cnt, kid = get_knn_distr_redundancy(gt, d2b, cfg)
    found = rng.integers(0, 300, (nq, nb, k))
    for i in range(nq):  # plant some true hits
        for g in gt[i][:3]:
            b = d2b[g, 0]
            found[i, b, 0] = g
    scores = rng.random((nq, nb))
    st = rng.random((nq, nb)) * 1e-3
    cmp_ = rng.integers(100, 200, (nq, nb))
    rows = query_tuning(scores, kid, found, st, cmp_, cfg)
    for row in rows[::7]:
        t = row["threshold"]
        rec, tm = [], []
        for i in range(nq):  # LIRA_smallscale.py:204-214
            probe = np.where(scores[i] > t)[0]
            fk = set()
            for b in probe:
                fk.update(set(kid[i][b]).intersection(found[i][b]))
            rec.append(len(fk) / k)
            tm.append(st[i, probe].sum())
        assert row["Recall"] == pytest.approx(np.mean(rec))
        assert row["QPS"] == pytest.approx(1.0 / np.mean(tm) if np.mean(tm) > 0 else 0.0)


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
def test_search_engine_nearest_probe_oracle(tmp_path, metric):
    """a scripted nearest-nprobe model + threshold 0.5 turns the
    search.cpp pipeline into exact IVF-nprobe; compare with the oracle."""
    from lira_amd.io import save_artifacts
    from lira_amd.probing import NearestCentroidProbe
    from lira_amd.search import SearchEngine
    x, c, rng = mixture(8000, 48, 16, 3)
    d2b = np.full((8000, 2), -1, np.int32)
    d2b[:, 0] = oracle.centroid_dist(x, c).argmin(1)
    d2b[:400, 1] = rng.integers(0, 16, 400)
    q = (c[rng.integers(0, 16, 100)] + 0.35 * rng.standard_normal((100, 48), dtype=np.float32)).astype(np.float32)
    prefix = str(tmp_path / "art")
    save_artifacts(prefix, c, d2b, x, np.zeros(16), np.ones(16), NearestCentroidProbe(4))
    eng = SearchEngine(prefix, metric)
    D, I, nprobe, ncand = eng.search(q, 0.5, 10)
    assert (nprobe.cpu().numpy() == 4).all()
    want_probe = np.sort(oracle.probe_nearest(oracle.centroid_dist(q, c), 4), axis=1)
    off, ids = oracle.build_csr(d2b, 16)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Do, Io, nco = oracle.scan_topk(q, off, ids, x[ids], want_probe, 10, met, 0)  # search.cpp keeps dups
    assert np.array_equal(I.cpu().numpy(), Io)
    assert np.array_equal(D.cpu().numpy().view(np.uint32), Do.view(np.uint32))
    assert np.array_equal(ncand.cpu().numpy(), nco)
    rows = eng.sweep(q, Io.astype(np.int32), 10, 0.5, 0.5, 0.02, verbose=False)
    assert rows[0]["avg_recall"] == 1.0


def test_search_engine_mlp_threshold():
    from lira_amd.io import save_artifacts
    from lira_amd.probing import MLP_2_Input
    from lira_amd.search import SearchEngine
    import tempfile
    x, c, rng = mixture(6000, 32, 12, 4)
    d2b = oracle.centroid_dist(x, c).argmin(1).astype(np.int32)[:, None]
    q = (c[rng.integers(0, 12, 80)] + 0.35 * rng.standard_normal((80, 32), dtype=np.float32)).astype(np.float32)
    dist = oracle.centroid_dist(x, c)
    mean, scale = dist.mean(0).astype(np.float32), dist.std(0).astype(np.float32)
    torch.manual_seed(0)
    model = MLP_2_Input(12, 32, 12)
    with tempfile.TemporaryDirectory() as td:
        save_artifacts(td + "/a", c, d2b, x, mean, scale, model)
        eng = SearchEngine(td + "/a")
    qt = torch.from_numpy(q).cuda()
    s = eng.scores(qt)
    # scores = the model on the exact standardised distances (search.cpp:427-445)
    want = model.cuda()(torch.from_numpy(oracle.centroid_dist(q, c, mean, scale)).cuda(), qt)
    assert torch.equal(s, want)
    thr = float(np.median(s.cpu().numpy()))
    D, I, nprobe, ncand = eng.search(qt, thr, 10, scores=s)
    pr, cnt = oracle.probe_threshold(s.cpu().numpy(), thr)
    assert np.array_equal(nprobe.cpu().numpy(), cnt)
    off, ids = oracle.build_csr(d2b, 12)
    Do, Io, _ = oracle.scan_topk(q, off, ids, x[ids], pr, 10, oracle.L2, 0)
    assert np.array_equal(I.cpu().numpy(), Io)


def test_probe_pipeline_graph_matches_eager_and_oracle():
    """The MLP-probed search.cpp pipeline (search.cpp:424-514) on preallocated
    buffers, eagerly and replayed from one captured HIP graph: identical to
    each other, and to the oracle given the pipeline's own scores."""
    from lira_amd import PartitionedIndex
    from lira_amd.probing import MLP_2_Input, fit_probe_to_nearest, standard_scaler
    from lira_amd.search import ProbePipeline
    from lira_amd import centroid_dist
    x, c, rng = mixture(20000, 32, 16, 7)
    d2b = oracle.centroid_dist(x, c).argmin(1).astype(np.int32)[:, None]
    dev = torch.device("cuda", 0)
    xt, ct = torch.from_numpy(x).to(dev), torch.from_numpy(c).to(dev)
    idx = PartitionedIndex.from_assignment(xt, torch.from_numpy(d2b).to(dev), 16, "L2")
    mean, scale = standard_scaler(centroid_dist(xt[:4096], ct))
    model = MLP_2_Input(16, 32, 16).to(dev)

    def batch(n, it):
        g = torch.Generator(device=dev).manual_seed(100 + it)
        qb = ct[torch.randint(0, 16, (n,), generator=g, device=dev)] + 0.35 * torch.randn(
            (n, 32), generator=g, device=dev)
        return centroid_dist(qb, ct, mean, scale), qb

    fit_probe_to_nearest(model, batch, 3, steps=60, batch=1024)
    q = (c[rng.integers(0, 16, 300)] + 0.35 * rng.standard_normal((300, 32), dtype=np.float32)).astype(np.float32)
    pipe = ProbePipeline(idx, ct, mean, scale, model, 300, 10, 0.5)
    pipe.q.copy_(torch.from_numpy(q))
    pipe.run()
    torch.cuda.synchronize()
    D0, I0, np0, s0 = pipe.D.clone(), pipe.I.clone(), pipe.nprobe.clone(), pipe.scores.clone()
    pipe.capture()
    pipe.D.zero_()
    pipe.I.zero_()
    pipe.replay()
    torch.cuda.synchronize()
    assert torch.equal(pipe.I, I0) and torch.equal(pipe.D.view(torch.int32), D0.view(torch.int32))
    assert torch.equal(pipe.nprobe, np0)
    # oracle: exact standardised distances, select on the pipeline's scores, scan
    dist_o = oracle.centroid_dist(q, c, mean.cpu().numpy(), scale.cpu().numpy())
    assert np.array_equal(pipe.dist.cpu().numpy().view(np.uint32), dist_o.view(np.uint32))
    pr, cnt = oracle.probe_threshold(s0.cpu().numpy(), 0.5)
    assert np.array_equal(np0.cpu().numpy(), cnt) and 1.0 <= cnt.mean() <= 16
    off, ids = oracle.build_csr(d2b, 16)
    Do, Io, _ = oracle.scan_topk(q, off, ids, x[ids], pr, 10, oracle.L2, 1)
    assert np.array_equal(I0.cpu().numpy(), Io)
    assert np.array_equal(D0.cpu().numpy().view(np.uint32), Do.view(np.uint32))
    # a run at another threshold drops the graph (its selection threshold is baked in)
    pipe.run(0.5)
    assert pipe.graph is not None
    pipe.run(0.3)
    assert pipe.graph is None
    with pytest.raises(RuntimeError, match="no captured graph"):
        pipe.replay()


def test_search_engine_results_do_not_alias():
    # SearchEngine.search returns fresh tensors (a later search of the same
    # shape does not overwrite them), reuses one pipeline across thresholds and
    # leaves the index's options as they were
    from lira_amd.io import save_artifacts
    from lira_amd.probing import MLP_2_Input
    from lira_amd.search import SearchEngine
    import tempfile
    x, c, rng = mixture(6000, 32, 12, 5)
    d2b = oracle.centroid_dist(x, c).argmin(1).astype(np.int32)[:, None]
    q = (c[rng.integers(0, 12, 64)] + 0.35 * rng.standard_normal((64, 32), dtype=np.float32)).astype(np.float32)
    dist = oracle.centroid_dist(x, c)
    torch.manual_seed(1)
    with tempfile.TemporaryDirectory() as td:
        save_artifacts(td + "/a", c, d2b, x, dist.mean(0).astype(np.float32), dist.std(0).astype(np.float32),
                       MLP_2_Input(12, 32, 12))
        eng = SearchEngine(td + "/a")
    qt = torch.from_numpy(q).cuda()
    s = eng.scores(qt).cpu().numpy()
    t1, t2 = float(np.quantile(s, 0.3)), float(np.quantile(s, 0.7))
    D1, I1, n1, _ = eng.search(qt, t1, 10)
    D1c, I1c, n1c = D1.clone(), I1.clone(), n1.clone()
    pipe = eng._pipe
    D2, I2, n2, _ = eng.search(qt, t2, 10)
    assert eng._pipe is pipe
    assert torch.equal(D1, D1c) and torch.equal(I1, I1c) and torch.equal(n1, n1c)
    assert not torch.equal(n1, n2)
    # each threshold's result equals a scan of its own selection
    for thr, I, n in ((t1, I1, n1), (t2, I2, n2)):
        pr, cnt = oracle.probe_threshold(s, thr)
        assert np.array_equal(n.cpu().numpy(), cnt)
    assert eng.index.get_option("probes_hint") == 0


@pytest.mark.parametrize("mp,nb", [(8, 16), (64, 64), (100, 130), (256, 300)])
def test_order_probes_matches_numpy(mp, nb):
    # lira_order_probes: each row's valid probes by ascending key (ties -> smaller
    # bucket), -1 slots last; the probe set is unchanged
    from lira_amd import order_probes
    rng = np.random.default_rng(mp + nb)
    n = 300
    key = rng.integers(0, 50, (n, nb)).astype(np.float32)  # many exact ties
    key[:, 3] = -0.0
    key[:, 5] = 0.0
    probe = np.full((n, mp), -1, np.int32)
    for i in range(n):
        m = int(rng.integers(0, min(mp, nb) + 1))
        probe[i, :m] = rng.permutation(nb)[:m]
        if i % 7 == 0 and m < mp:  # an out-of-range id: kept (after the valid ones) for the scan's ERANGE
            probe[i, m] = nb + i % 5
        rng.shuffle(probe[i])  # -1 slots anywhere
    got = order_probes(torch.from_numpy(probe).cuda(), torch.from_numpy(key).cuda()).cpu().numpy()
    for i in range(n):
        v = probe[i][(probe[i] >= 0) & (probe[i] < nb)]
        kk = key[i, v] + np.float32(0.0)  # (-0 orders as +0)
        want = np.concatenate([v[np.lexsort((v, kk))], np.sort(probe[i][probe[i] >= nb])])
        assert np.array_equal(got[i, :len(want)], want) and (got[i, len(want):] == -1).all()
