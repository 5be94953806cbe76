"""GPU parity: query->centroid ranking (exact distances, MFMA GEMM with the
exact boundary re-check) and probe selection against the oracle."""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("name", ["toy_l2", "sift_like_redundant", "deep_like_k100_ip", "odd_dim"])
def test_centroid_dist_golden(name):
    from lira_amd import centroid_dist
    g = load_golden(name)
    q = torch.from_numpy(g["q"]).cuda()
    c = torch.from_numpy(g["centroids"]).cuda()
    out = centroid_dist(q, c).cpu().numpy()
    assert np.array_equal(bits(out), bits(g["qdist"]))  # search.cpp:220-235
    out = centroid_dist(q, c, torch.from_numpy(g["scaler_mean"]), torch.from_numpy(g["scaler_scale"]))
    assert np.array_equal(bits(out.cpu().numpy()), bits(g["qdist_std"]))  # :238-250


@pytest.mark.parametrize("nq,nb,d", [(1, 8, 16), (100, 64, 128), (257, 130, 96), (33, 1024, 128),
                                     (16, 128, 960), (70, 5, 7),
                                     # the one-pass exact kernel (nb <= 64, d % 4 == 0, d <= 256):
                                     # several workgroups with a partial last one, the LDS maximum
                                     (1000, 64, 256), (65, 33, 100), (300, 64, 132), (37, 64, 260),
                                     # the chunked one-pass kernel (nb <= 256, d % 4 == 0): 2 and 4
                                     # centroids per lane, 4- and 8-wave workgroups, several dim chunks
                                     (4100, 256, 96), (4097, 200, 64), (3, 250, 1000), (129, 65, 512)])
def test_gemm_bound_and_rank_nearest(nq, nb, d):
    from lira_amd import centroid_dist, centroid_gemm, rank_nearest, select_probes
    rng = np.random.default_rng(nq * 7 + nb)
    c = rng.standard_normal((nb, d), dtype=np.float32)
    q = (c[rng.integers(0, nb, nq)] + 0.3 * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
    qt, ct = torch.from_numpy(q).cuda(), torch.from_numpy(c).cuda()
    A, err = centroid_gemm(qt, ct)
    exact = oracle.centroid_dist(q, c).astype(np.float64) ** 2
    A = A.cpu().numpy().astype(np.float64)
    err = err.cpu().numpy().astype(np.float64)
    assert (np.abs(A - exact) <= err[:, None] + 1e-6 * exact).all()
    # relative accuracy of the MFMA GEMM itself (fp32, ~1e-5 with cancellation)
    assert np.allclose(A, exact, rtol=1e-3, atol=1e-3 * exact.mean())
    for nprobe in sorted({1, min(8, nb), min(32, nb), min(nb, 64), min(nb + 3, 256)}):
        got = rank_nearest(qt, ct, nprobe).cpu().numpy()
        want = oracle.probe_nearest(oracle.centroid_dist(q, c), nprobe)
        assert np.array_equal(got, want)
        sel, cnt = select_probes(centroid_dist(qt, ct), "nearest", nprobe)
        assert np.array_equal(sel.cpu().numpy(), want)


def test_rank_nearest_ties_and_duplicates():
    from lira_amd import rank_nearest
    # duplicated centroids -> exact ties broken by smaller bucket id
    rng = np.random.default_rng(2)
    base = rng.standard_normal((8, 32), dtype=np.float32)
    c = np.concatenate([base, base, base[:3]])
    q = rng.standard_normal((40, 32), dtype=np.float32)
    got = rank_nearest(torch.from_numpy(q).cuda(), torch.from_numpy(c).cuda(), 6).cpu().numpy()
    want = oracle.probe_nearest(oracle.centroid_dist(q, c), 6)
    assert np.array_equal(got, want)
    # integer-valued (SIFT-like) data: many exactly equal distances
    c = rng.integers(0, 4, (64, 16)).astype(np.float32)
    q = rng.integers(0, 4, (50, 16)).astype(np.float32)
    got = rank_nearest(torch.from_numpy(q).cuda(), torch.from_numpy(c).cuda(), 8).cpu().numpy()
    assert np.array_equal(got, oracle.probe_nearest(oracle.centroid_dist(q, c), 8))


@pytest.mark.parametrize("thr", [0.02, 0.3, 0.5, 0.8, 1.5])
def test_threshold_select(thr):
    from lira_amd import select_probes
    rng = np.random.default_rng(int(thr * 100))
    s = rng.random((300, 70), dtype=np.float32)
    s[5] = 0.1  # all below: argmax fallback picks bucket 0 (first max)
    s[6, 3] = s[6, 9] = 0.95
    s[6, :3] = 0.0
    s[6, 4:9] = 0.0
    s[6, 10:] = 0.0
    for mode, strict in (("ge", False), ("gt", True)):
        p, c = select_probes(torch.from_numpy(s).cuda(), mode, 70, thr)
        wp, wc = oracle.probe_threshold(s, thr, strict)
        assert np.array_equal(c.cpu().numpy(), wc)
        assert np.array_equal(p.cpu().numpy(), wp)
    # truncation at max_probe keeps the first (ascending-bucket) entries
    p, c = select_probes(torch.from_numpy(s).cuda(), "ge", 4, thr)
    wp, wc = oracle.probe_threshold(s, thr, False)
    assert np.array_equal(p.cpu().numpy(), wp[:, :4])
    assert np.array_equal(c.cpu().numpy(), np.minimum(wc, 4))


@pytest.mark.parametrize("thr", [0.3, 0.8, 1.5])
def test_threshold_select_by_score(thr):
    # LIRA_PROBE_BY_SCORE: search.cpp's set, descending score (ties -> smaller
    # bucket); truncation keeps the highest scores; argmax fallback as before
    from lira_amd import select_probes
    rng = np.random.default_rng(int(thr * 10) + 7)
    s = np.round(rng.random((200, 150), dtype=np.float32) * 20) / 20  # many exact ties
    s[3] = 0.1
    for mode, strict in (("ge", False), ("gt", True)):
        for maxp in (150, 5):
            p, c = select_probes(torch.from_numpy(s).cuda(), mode, maxp, thr, by_score=True)
            p, c = p.cpu().numpy(), c.cpu().numpy()
            wp, wc = oracle.probe_threshold(s, thr, strict)
            assert np.array_equal(c, np.minimum(wc, maxp))
            for i in range(s.shape[0]):
                sel = wp[i][wp[i] >= 0]
                want = sorted(sel, key=lambda b: (-s[i, b], b))[:maxp]
                assert list(p[i][:c[i]]) == want and (p[i][c[i]:] == -1).all()
