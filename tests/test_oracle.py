"""CPU: the oracle restatement against the golden fixtures, the reference's own
compiled functions (when built here) and plain-numpy restatements."""
import numpy as np
import pytest

import oracle
from conftest import load_golden


def test_fixtures_were_pinned_by_reference(golden_names):
    assert golden_names, "tests/golden holds no fixtures"
    for n in golden_names:
        assert bool(load_golden(n)["ref_pinned"]), f"{n} was not checked against search.cpp"


@pytest.mark.parametrize("name", ["toy_l2", "toy_ip", "sift_like_redundant", "deep_like_k100_ip",
                                  "odd_dim"])
def test_oracle_reproduces_golden(name):
    g = load_golden(name)
    met = oracle.IP if str(g["metric"]) == "inner_product" else oracle.L2
    n_bkt = g["centroids"].shape[0]
    off, ids = oracle.build_csr(g["data_2_bkt"], n_bkt)
    assert np.array_equal(off, g["offsets"]) and np.array_equal(ids, g["ids"])
    vecs = oracle.gather_lists(g["x"], off, ids)
    k = int(g["k"])
    D, I, nc = oracle.scan_topk(g["q"], off, ids, vecs, g["probe"], k, met, int(g["dedup_rep"]))
    assert np.array_equal(D.view(np.uint32), g["D"].view(np.uint32))
    assert np.array_equal(I, g["I"]) and np.array_equal(nc, g["ncand"])
    Dp, Ip = oracle.scan_per_partition(g["q"], off, ids, vecs, g["probe"], k, met)
    assert np.array_equal(Dp.view(np.uint32), g["D_part"].view(np.uint32))
    assert np.array_equal(Ip, g["I_part"])
    qd = oracle.centroid_dist(g["q"], g["centroids"])
    assert np.array_equal(qd.view(np.uint32), g["qdist"].view(np.uint32))
    qs = oracle.centroid_dist(g["q"], g["centroids"], g["scaler_mean"], g["scaler_scale"])
    assert np.array_equal(qs.view(np.uint32), g["qdist_std"].view(np.uint32))


def test_oracle_against_reference_binary():
    R = oracle.ref()
    if R is None:
        pytest.skip("oracle/_ref/libref_search.so not built (needs /root/reference)")
    rng = np.random.default_rng(5)
    for d in (1, 3, 16, 96, 128, 960):
        for _ in range(50):
            a = (rng.standard_normal(d) * rng.uniform(0.01, 300)).astype(np.float32)
            b = rng.standard_normal(d).astype(np.float32)
            r = np.float32(R.ref_l2_sq(a.ctypes.data, b.ctypes.data, d))
            assert r.view(np.uint32) == oracle.l2_sq(a, b).view(np.uint32)
            r = np.float32(R.ref_ip(a.ctypes.data, b.ctypes.data, d))
            assert r.view(np.uint32) == oracle.ip(a, b).view(np.uint32)


def test_l2_matches_sequential_numpy():
    rng = np.random.default_rng(1)
    for d in (1, 5, 64, 129):
        a = rng.standard_normal(d).astype(np.float32) * 50
        b = rng.standard_normal(d).astype(np.float32)
        assert oracle.l2_sq(a, b).view(np.uint32) == oracle.l2_sq_np(a, b).view(np.uint32)


def test_build_csr_semantics():
    # search.cpp:371-385: -1 skipped, duplicate bucket in one row collapsed, sorted
    d2b = np.array([[2, -1], [0, 2], [2, 2], [1, -1], [0, -1]], dtype=np.int32)
    off, ids = oracle.build_csr(d2b, 4)
    assert off.tolist() == [0, 2, 3, 6, 6]
    assert ids.tolist() == [1, 4, 3, 0, 1, 2]
    with pytest.raises(RuntimeError):
        oracle.build_csr(np.array([[4]], dtype=np.int32), 4)


def test_probe_threshold_semantics():
    s = np.array([[0.1, 0.7, 0.7, 0.2], [0.1, 0.3, 0.3, 0.2], [0.5, 0.5, 0.9, 0.5]], np.float32)
    p, c = oracle.probe_threshold(s, 0.5)  # >= with argmax fallback (search.cpp:447-466)
    assert c.tolist() == [2, 1, 4]
    assert p[0, :2].tolist() == [1, 2] and p[1, 0] == 1  # first max wins
    assert p[2].tolist() == [0, 1, 2, 3]
    p, c = oracle.probe_threshold(s, 0.5, strict=True)  # LIRA_smallscale.py:206
    assert c.tolist() == [2, 0, 1] and p[1, 0] == -1


def test_probe_nearest_ties():
    d = np.array([[3.0, 1.0, 1.0, 0.5, 1.0]], np.float32)
    assert oracle.probe_nearest(d, 3).tolist() == [[3, 1, 2]]
    assert oracle.probe_nearest(d, 7).tolist() == [[3, 1, 2, 4, 0, -1, -1]]


def test_scan_dedup_and_padding():
    # one vector in two buckets, both probed: reference multiset keeps it twice
    x = np.array([[0, 0], [1, 0], [5, 5]], np.float32)
    d2b = np.array([[0, 1], [0, -1], [1, -1]], np.int32)
    off, ids = oracle.build_csr(d2b, 2)
    vecs = oracle.gather_lists(x, off, ids)
    q = np.zeros((1, 2), np.float32)
    probe = np.array([[0, 1]], np.int32)
    D, I, nc = oracle.scan_topk(q, off, ids, vecs, probe, 3, oracle.L2, 0)
    assert I.tolist() == [[0, 0, 1]] and nc.tolist() == [4]
    D, I, nc = oracle.scan_topk(q, off, ids, vecs, probe, 4, oracle.L2, 2)
    assert I.tolist() == [[0, 1, 2, -1]] and np.isinf(D[0, 3])
    D, I, _ = oracle.scan_topk(q, off, ids, vecs, probe, 2, oracle.IP, 2)
    assert D.dtype == np.float32 and I[0, 0] in (0, 1)


def test_recall_definition():
    # search.cpp:519-528
    r = oracle.recall_at_k(np.array([[1, 2, 3, -1]]), np.array([[3, 9, 1, 2]]), 2)
    assert r.tolist() == [0.5]
