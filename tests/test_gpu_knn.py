"""GPU: offline self-kNN (compute_knn.cpp / utils.compute_data_knn) and the
k-means assignment (utils.py:321-330) on the HIP kernels, against the oracle."""
import os
import types

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def mixture(seed, n, d, b):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((b, d), dtype=np.float32)
    return (c[rng.integers(0, b, n)] + 0.35 * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)


def oracle_self_knn(x, k, met):
    n = x.shape[0]
    off = np.array([0, n], np.int64)
    ids = np.arange(n, dtype=np.int32)
    probe = np.zeros((n, 1), np.int32)
    D, I, _ = oracle.scan_topk(x, off, ids, x, probe, k + 1, met, 0)
    return D[:, 1:], I[:, 1:]


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
def test_exact_self_knn_matches_oracle(metric):
    from lira_amd.knn import self_knn
    x = mixture(5, 3000, 24, 8)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Do, Io = oracle_self_knn(x, 10, met)
    I, D = self_knn(x, 10, metric, batch_size=1000, return_distances=True)
    assert I.dtype == np.int32 and I.shape == (3000, 10)
    assert np.array_equal(I, Io.astype(np.int32))
    assert np.array_equal(D.view(np.uint32), Do.view(np.uint32))
    if metric == "L2":  # the dropped first neighbour is the row itself (distinct rows)
        Ifull = self_knn(x, 1, metric)
        assert (Ifull[:, 0] != np.arange(3000)).all()


def test_kmeans_assign_is_exact_nearest_centroid():
    from lira_amd.knn import kmeans_assign
    x = mixture(6, 5000, 32, 16)
    c = mixture(7, 40, 32, 16)
    a = kmeans_assign(x, c).cpu().numpy()
    assert np.array_equal(a, oracle.probe_nearest(oracle.centroid_dist(x, c), 1))


def test_kmeans_and_ivf_self_knn():
    from lira_amd.knn import Kmeans, build_kmeans_index, self_knn
    x = mixture(8, 20000, 16, 12)
    km = Kmeans(16, 12, niter=10)
    km.train(x)
    assert km.centroids.shape == (12, 16)
    _, lab = km.index.search(x, 1)
    cnt = np.bincount(lab[:, 0], minlength=12)
    assert (cnt > 0).all()
    # Lloyd's objective does not increase between a fresh and a trained model
    km0 = Kmeans(16, 12, niter=0)
    km0.train(x)
    def obj(cs):
        return float(((x - cs[np.asarray(oracle.probe_nearest(oracle.centroid_dist(x, cs), 1))[:, 0]]) ** 2).sum())
    assert obj(km.centroids) <= obj(km0.centroids)
    kmi, d2b, cnts, cluster_ids = build_kmeans_index(x, 12, niter=5)
    assert d2b.shape == (20000, 1) and cnts.sum() == 20000
    assert sorted(i for c in cluster_ids for i in c) == list(range(20000))
    assert all(d2b[i, 0] == b for b, c in enumerate(cluster_ids) for i in c[:5])
    # IVF-approximate self-kNN: high recall against the exact one
    exact = self_knn(x, 10, nprobe=0)
    approx = self_knn(x, 10, nprobe=-1, niter=10)
    rec = np.mean([len(set(a) & set(e)) / 10 for a, e in zip(approx[:2000], exact[:2000])])
    assert rec > 0.9


def test_cli_writes_compute_knn_file(tmp_path):
    from lira_amd.io import write_xvecs
    from lira_amd.knn import main, self_knn
    x = mixture(9, 2000, 8, 4)
    os.makedirs(tmp_path / "toy")
    write_xvecs(str(tmp_path / "toy" / "toy_base.fvecs"), x)
    assert main(["toy", str(tmp_path), "5", "0"]) == 0
    f = tmp_path / "toy" / "knn_cache" / "toy-data_self_knn5-n2000.bin"
    got = np.fromfile(f, dtype=np.int32).reshape(2000, 5)
    assert np.array_equal(got, self_knn(x, 5))
    assert main(["missing", str(tmp_path), "5"]) == 1
