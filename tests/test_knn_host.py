"""CPU: the self-kNN host contract of compute_knn.cpp / utils.compute_data_knn
(parameters, file names, cache lookup) -- no GPU needed."""
import os
import types

import numpy as np
import pytest

from lira_amd.knn import compute_data_knn, ivf_params, knn_cache_name


@pytest.mark.parametrize("n,nprobe,expect", [
    (10_000, -1, (100, 25)),        # n < 50k: sqrt capped 256; auto nprobe = clamp(n_list/4, 16, 64)
    (40_000, -1, (200, 50)),
    (60_000, -1, (244, 61)),        # 50k <= n < 1M: cap 1024
    (500_000, -1, (707, 88)),       # n >= 100k: clamp(n_list/8, 32, 128)
    (1_000_000, -1, (1000, 125)),   # n >= 1M: cap 4096
    (4_000_000, -1, (2000, 128)),
    (1_000_000, 64, (1000, 64)),
    (100, 300, (10, 10)),           # explicit nprobe is clamped to n_list
])
def test_ivf_params_follow_compute_knn(n, nprobe, expect):
    assert ivf_params(n, nprobe) == expect


def test_cache_names():
    assert knn_cache_name("sift", 10, 1000000) == "sift-data_self_knn10-n1000000.bin"
    assert knn_cache_name("sift", 10, 1000000, 64) == "sift-data_self_knn10-n1000000_ivf_nprobe64.bin"


def test_compute_data_knn_prefers_cpp_cache(tmp_path):
    cfg = types.SimpleNamespace(dataset="toy", k=3, dis_metric="L2")
    x = np.zeros((5, 4), np.float32)
    d = tmp_path / "toy" / "knn_cache"
    d.mkdir(parents=True)
    exact = np.arange(15, dtype=np.int32).reshape(5, 3)
    exact.tofile(d / "toy-data_self_knn3-n5.bin")
    np.save(d / "toy-data_self_knn3-n5.npy", exact + 100)
    assert np.array_equal(compute_data_knn(x, cfg, str(tmp_path)), exact)   # .bin before .npy
    ivf = exact + 7
    ivf.tofile(d / "toy-data_self_knn3-n5_ivf_nprobe4.bin")
    assert np.array_equal(compute_data_knn(x, cfg, str(tmp_path)), ivf)     # IVF cache first
    for f in os.listdir(d):
        if f.endswith(".bin"):
            os.remove(d / f)
    assert np.array_equal(compute_data_knn(x, cfg, str(tmp_path)), exact + 100)
