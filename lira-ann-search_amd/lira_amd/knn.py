"""Offline exhaustive self-kNN and k-means assignment on the HIP scan
(SURVEY.md 8(f) row 4).

Replaces, with the same inputs, outputs and on-disk contract:

* ``compute_knn.cpp`` (the ``compute_knn <dataset> <data_path> <k> [nprobe]
  [n_threads]`` program, compute_knn.cpp:60-307): self-kNN of the base set,
  exact (nprobe = 0, FLAT) or IVF-approximate (nprobe != 0, n_list and the
  auto nprobe from compute_knn.cpp:150-196), k+1 neighbours per row with the
  first column dropped (compute_knn.cpp:240-251), written as a raw int32
  ``{ds}-data_self_knn{k}-n{n}[_ivf_nprobe{p}].bin`` under ``knn_cache``.
* ``compute_data_knn`` (utils.py:222-319): same cache lookup order (.bin from
  the C++ tool, then .npy), then an exact search in the dataset's metric.
* ``build_kmeans_index`` / ``faiss.Kmeans`` (utils.py:321-330): Lloyd
  iterations whose assignment step is the exact nearest-centroid ranking
  (lira_rank_nearest); ``kmeans.index.search(x, 1)`` is the exact scan.

The distance arithmetic is the scan's (search.cpp:253-269 order).  faiss is not
available here, so k-means centroids are not comparable with faiss's (its RNG
and sampling are its own): the assignment and the kNN scan are the pinned
parts (tests/test_gpu_knn.py), the clustering itself is parity unpinned.
"""
from __future__ import annotations

import glob
import math
import os
import sys
import time

import numpy as np
import torch

from .faiss_compat import IndexFlat
from .index import PartitionedIndex, normalize_metric, rank_nearest


def _as_cuda(x, device=None) -> torch.Tensor:
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.float32).contiguous()
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev)


# ------------------------------------------------------------------ k-means
class Kmeans:
    """GPU Lloyd k-means with faiss.Kmeans' interface (d, k, niter, seed,
    max_points_per_centroid; ``train``; ``centroids``; ``index``).

    Init: k distinct training points drawn with ``seed``; training set
    subsampled to k * max_points_per_centroid as faiss does; an empty
    cluster takes a copy of the largest one, both nudged by +-1/1024
    (faiss's split rule).  Assignment: exact nearest centroid (L2 always,
    as utils.py:323 and search.cpp:427 rank with L2)."""

    def __init__(self, d: int, k: int, niter: int = 25, seed: int = 1234,
                 max_points_per_centroid: int = 256, verbose: bool = False, device=None):
        self.d, self.k, self.niter, self.seed = int(d), int(k), int(niter), int(seed)
        self.max_points_per_centroid = int(max_points_per_centroid)
        self.verbose = verbose
        self.device = device
        self.centroids: np.ndarray | None = None
        self.obj: list[float] = []
        self.index: IndexFlat | None = None

    def train(self, x) -> float:
        xt = _as_cuda(x, self.device)
        n = xt.shape[0]
        if xt.dim() != 2 or xt.shape[1] != self.d:
            raise RuntimeError(f"train: expected (n, {self.d}) vectors")
        if n < self.k:
            raise RuntimeError(f"Number of training points ({n}) should be at least "
                               f"as large as number of clusters ({self.k})")
        g = np.random.default_rng(self.seed)
        cap = self.k * self.max_points_per_centroid
        if n > cap:
            sel = torch.from_numpy(np.sort(g.choice(n, cap, replace=False))).to(xt.device)
            xt = xt.index_select(0, sel)
            n = cap
        c = xt.index_select(0, torch.from_numpy(g.choice(n, self.k, replace=False)).to(xt.device)).clone()
        eps = 1.0 / 1024
        for it in range(self.niter):
            a = rank_nearest(xt, c, 1)[:, 0].to(torch.int64)
            cnt = torch.bincount(a, minlength=self.k)
            s = torch.zeros_like(c).index_add_(0, a, xt)
            nz = cnt > 0
            c[nz] = s[nz] / cnt[nz, None].to(torch.float32)
            empty = torch.nonzero(~nz).flatten().tolist()
            if empty:
                cnt_h = cnt.cpu().numpy().astype(np.float64)
                for ci in empty:  # split the largest cluster (faiss clustering.cpp)
                    cj = int(np.argmax(cnt_h))
                    c[ci] = c[cj] * (1 + eps)
                    c[cj] = c[cj] * (1 - eps)
                    cnt_h[ci] = cnt_h[cj] / 2
                    cnt_h[cj] -= cnt_h[ci]
            if self.verbose:
                print(f"  Iteration {it} ({len(empty)} splits)", file=sys.stderr)
        self.centroids = c.cpu().numpy()
        self.index = IndexFlat(self.d, "L2", xt.device.index)
        self.index.add(c)
        return 0.0


def kmeans_assign(x, centroids, nprobe: int = 1) -> torch.Tensor:
    """``kmeans.index.search(x, 1)`` labels (utils.py:325): nearest centroid by
    the exact search.cpp distance (ties -> smaller id), (n, nprobe) int32."""
    xt = _as_cuda(x)
    return rank_nearest(xt, _as_cuda(centroids, xt.device.index), nprobe)


def build_kmeans_index(x_data, n_bkt: int, niter: int = 20, seed: int = 1234):
    """utils.py:321-330: (kmeans, data_2_bkt (n,1) int64, cluster_cnts, cluster_ids)."""
    x = _as_cuda(x_data)
    km = Kmeans(x.shape[1], n_bkt, niter=niter, seed=seed)
    km.train(x)
    _, d2b = km.index.search(x, 1)
    d2b = d2b.cpu().numpy()
    cnts = np.bincount(d2b.flatten(), minlength=n_bkt)
    order = np.argsort(d2b[:, 0], kind="stable")
    cluster_ids = [list(map(int, s)) for s in np.split(order, np.cumsum(cnts)[:-1])]
    return km, d2b, cnts, cluster_ids


# ---------------------------------------------------------------- self-kNN
def ivf_params(n: int, nprobe: int) -> tuple[int, int]:
    """n_list and the effective nprobe of compute_knn.cpp:150-196 (nprobe < 0 = auto)."""
    if n < 50000:
        n_list = min(int(math.sqrt(n)), 256)
    elif n < 1000000:
        n_list = min(int(math.sqrt(n)), 1024)
    else:
        n_list = min(int(math.sqrt(n)), 4096)
    if nprobe < 0:
        nprobe = min(max(n_list // 4, 16), 64) if n < 100000 else min(max(n_list // 8, 32), 128)
    return n_list, min(nprobe, n_list)


def self_knn(x, k: int, metric: str = "L2", nprobe: int = 0, batch_size: int = 32768,
             niter: int = 25, seed: int = 1234, return_distances: bool = False):
    """Self-kNN of x: search k+1 neighbours of every row among all rows and
    drop column 0 (compute_knn.cpp:240-251, utils.py:303-307 -- the first
    neighbour is taken to be the row itself, as both do).

    nprobe == 0: exact (one list holding every row).  nprobe != 0: IVF over
    k-means lists (n_list from ivf_params), the nprobe nearest lists per row,
    nprobe < 0 picks compute_knn.cpp's auto value.
    Returns (n, k) int32 numpy (and the (n, k) float32 distances if asked).
    """
    metric = normalize_metric(metric)
    xt = _as_cuda(x)
    n, d = xt.shape
    idx = PartitionedIndex(d, metric, xt.device.index)
    cent = None
    if nprobe == 0:
        idx.add_lists(np.array([0, n], dtype=np.int64),
                      torch.arange(n, dtype=torch.int32, device=xt.device), xt, 1)
        n_probe = 1
    else:
        n_list, n_probe = ivf_params(n, nprobe)
        km = Kmeans(d, n_list, niter=niter, seed=seed, device=xt.device.index)
        km.train(xt)
        cent = torch.from_numpy(km.centroids).to(xt.device)
        assign = kmeans_assign(xt, cent, 1)
        idx.build(assign, xt, n_list)
    labels = np.empty((n, k), dtype=np.int32)
    dists = np.empty((n, k), dtype=np.float32) if return_distances else None
    for s in range(0, n, batch_size):
        e = min(n, s + batch_size)
        qb = xt[s:e]
        if cent is None:
            probe = torch.zeros((e - s, 1), dtype=torch.int32, device=xt.device)
        else:
            probe = rank_nearest(qb, cent, n_probe)
        D, I, _ = idx.search(qb, probe, k + 1)
        labels[s:e] = I[:, 1:].to(torch.int32).cpu().numpy()
        if dists is not None:
            dists[s:e] = D[:, 1:].cpu().numpy()
    idx.close()
    return (labels, dists) if return_distances else labels


def knn_cache_name(dataset: str, k: int, n: int, nprobe: int = 0) -> str:
    """compute_knn.cpp:255-259 output name."""
    suffix = f"_ivf_nprobe{nprobe}" if nprobe != 0 else ""
    return f"{dataset}-data_self_knn{k}-n{n}{suffix}.bin"


def compute_data_knn(x_data, cfg, data_path: str = "/data/vector_datasets") -> np.ndarray:
    """utils.py:222-319: load the C++ .bin cache (IVF first, then exact), then
    the .npy cache, else compute exactly in cfg.dis_metric and cache as .npy."""
    cache_dir = os.path.join(data_path, cfg.dataset, "knn_cache")
    os.makedirs(cache_dir, exist_ok=True)
    n = len(x_data)
    for pat in (f"{cfg.dataset}-data_self_knn{cfg.k}-n{n}_ivf_nprobe*.bin",
                f"{cfg.dataset}-data_self_knn{cfg.k}-n{n}.bin"):
        hits = glob.glob(os.path.join(cache_dir, pat))
        if hits:
            f = max(hits, key=os.path.getctime)
            return np.fromfile(f, dtype=np.int32).reshape(n, cfg.k)
    npy = os.path.join(cache_dir, f"{cfg.dataset}-data_self_knn{cfg.k}-n{n}.npy")
    if os.path.exists(npy):
        return np.load(npy).astype(int)
    knn = self_knn(x_data, cfg.k, getattr(cfg, "dis_metric", "L2"), nprobe=0)
    np.save(npy, knn)
    return knn


def main(argv=None) -> int:
    """``python -m lira_amd.knn <dataset_name> <data_path> <k> [nprobe] [n_threads]``
    (compute_knn.cpp:60-307; n_threads is accepted and ignored: the scan runs
    on the GPU)."""
    from .io import read_bvecs, read_fvecs
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 3:
        print("Usage: python -m lira_amd.knn <dataset_name> <data_path> <k> [nprobe] [n_threads]")
        print("  nprobe: number of clusters to probe (default: auto, 0=exact search)")
        return 1
    ds, path, k = argv[0], argv[1], int(argv[2])
    nprobe = int(argv[3]) if len(argv) > 3 else -1
    ddir = os.path.join(path, ds)
    base = os.path.join(ddir, f"{ds}_base.fvecs")
    try:
        if os.path.exists(base):
            x = read_fvecs(base)
        elif os.path.exists(os.path.join(ddir, f"{ds}_base.bvecs")):
            x = read_bvecs(os.path.join(ddir, f"{ds}_base.bvecs")).astype(np.float32)
        else:
            print(f"Error: Cannot find base file for dataset {ds}", file=sys.stderr)
            return 1
        n = x.shape[0]
        eff = 0 if nprobe == 0 else ivf_params(n, nprobe)[1]
        t0 = time.time()
        knn = self_knn(x, k, "L2", nprobe=nprobe)
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"Search time: {dt:.3f}s ({dt / max(n, 1) * 1000:.4f} ms/query)")
        out_dir = os.path.join(ddir, "knn_cache")
        os.makedirs(out_dir, exist_ok=True)
        out = os.path.join(out_dir, knn_cache_name(ds, k, n, eff))
        knn.astype(np.int32).tofile(out)
        print(f"Saved KNN results to: {out}\n  Shape: ({n}, {k})")
        return 0
    except Exception as e:  # compute_knn exits 1 on errors
        print(f"Error: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
