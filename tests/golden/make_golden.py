"""Generate the golden fixtures in tests/golden/*.npz.

Inputs are seeded Gaussian mixtures; expected outputs come from the CPU oracle
(oracle/lira_oracle.c, the restatement of search.cpp:220-514).  When the
reference's own compiled search.cpp functions are available
(oracle/_ref/libref_search.so, built by `make -C oracle ref` from
/root/reference), every distance the fixtures hold is also recomputed by the
reference code and must match bit for bit before anything is written; the
fixtures record that they were pinned ("ref_pinned").

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def mixture(n, d, b, seed, sigma=0.35):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((b, d), dtype=np.float32)
    lab = rng.integers(0, b, size=n)
    x = (c[lab] + np.float32(sigma) * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    return x, c


def pin_distances(q, x, ids, metric):
    """Recompute oracle distances with the reference's compiled l2_sq / ip."""
    R = oracle.ref()
    if R is None:
        return False
    f = R.ref_ip if metric == oracle.IP else R.ref_l2_sq
    of = oracle.ip if metric == oracle.IP else oracle.l2_sq
    for qi in range(q.shape[0]):
        qq = np.ascontiguousarray(q[qi])
        for g in ids[qi]:
            if g < 0:
                continue
            v = np.ascontiguousarray(x[g])
            a = np.float32(f(qq.ctypes.data, v.ctypes.data, len(qq)))
            b = of(qq, v)
            assert a.view(np.uint32) == b.view(np.uint32), (qi, g, a, b)
    return True


def pin_centroids(q, c, mean, scale, dist):
    R = oracle.ref()
    if R is None:
        return False
    out = np.empty(c.shape[0], dtype=np.float32)
    for qi in range(q.shape[0]):
        qq = np.ascontiguousarray(q[qi])
        R.ref_centroid_dist(qq.ctypes.data, c.ctypes.data, c.shape[0], c.shape[1],
                            None if mean is None else mean.ctypes.data,
                            None if scale is None else scale.ctypes.data, out.ctypes.data)
        assert np.array_equal(out.view(np.uint32), dist[qi].view(np.uint32)), qi
    return True


def case(name, n, d, b, nq, nprobe, k, metric, seed, redundancy=0.0, dedup=True):
    x, c = mixture(n, d, b, seed)
    q, _ = mixture(nq, d, b, seed + 1)
    rng = np.random.default_rng(seed + 2)
    # nearest-centre assignment (+ a second bucket for a `redundancy` fraction,
    # as LIRA's mul_partition_by_model does for its top rows)
    dist_x = oracle.centroid_dist(x, c)
    d2b = np.full((n, 2), -1, dtype=np.int32)
    d2b[:, 0] = dist_x.argmin(1)
    nred = int(n * redundancy)
    if nred:
        rows = rng.choice(n, nred, replace=False)
        second = np.argsort(dist_x[rows], axis=1)[:, 1]
        d2b[rows, 1] = second
    offsets, ids = oracle.build_csr(d2b, b)
    vecs = oracle.gather_lists(x, offsets, ids)
    # scaler as utils.get_scaled_dist fits it (StandardScaler over data distances)
    mean = dist_x.mean(0).astype(np.float32)
    scale = dist_x.std(0).astype(np.float32)
    scale[0] = 0.0  # exercise search.cpp:247 (scale 0 -> 1)
    qdist = oracle.centroid_dist(q, c)
    qdist_std = oracle.centroid_dist(q, c, mean, scale)
    probe = oracle.probe_nearest(qdist, nprobe)
    probe[0, -1] = -1  # a padded slot
    met = oracle.IP if metric == "inner_product" else oracle.L2
    rep = 2 if redundancy else 1
    D, I, nc = oracle.scan_topk(q, offsets, ids, vecs, probe, k, met, rep if dedup else 0)
    Dn, In, _ = oracle.scan_topk(q, offsets, ids, vecs, probe, k, met, 0)
    Dp, Ip = oracle.scan_per_partition(q, offsets, ids, vecs, probe, k, met)
    thr_probe, thr_cnt = oracle.probe_threshold(-qdist_std, 0.5)
    pinned = pin_distances(q, x, I, met) & pin_distances(q, x, In, met) & \
        pin_centroids(q, c, None, None, qdist) & pin_centroids(q, c, mean, scale, qdist_std)
    np.savez_compressed(
        os.path.join(OUT, f"{name}.npz"),
        x=x, centroids=c, q=q, data_2_bkt=d2b, offsets=offsets, ids=ids, probe=probe,
        scaler_mean=mean, scaler_scale=scale, qdist=qdist, qdist_std=qdist_std,
        k=np.int64(k), metric=np.array(metric), dedup_rep=np.int64(rep if dedup else 0),
        D=D, I=I, ncand=nc, D_nodedup=Dn, I_nodedup=In, D_part=Dp, I_part=Ip,
        thr_probe=thr_probe, thr_cnt=thr_cnt, ref_pinned=np.bool_(pinned),
    )
    print(f"{name}: n={n} d={d} B={b} nq={nq} nprobe={nprobe} k={k} {metric} "
          f"lists={np.diff(offsets).tolist()[:8]}... ref_pinned={pinned}")


if __name__ == "__main__":
    oracle.build()
    case("toy_l2", 4000, 16, 8, 64, 3, 10, "L2", 11)
    case("toy_ip", 4000, 16, 8, 64, 3, 10, "inner_product", 12)
    case("sift_like_redundant", 6000, 128, 16, 48, 4, 10, "L2", 13, redundancy=0.1)
    case("deep_like_k100_ip", 5000, 96, 32, 32, 6, 100, "inner_product", 14, redundancy=0.05)
    case("odd_dim", 3000, 7, 5, 40, 2, 17, "L2", 15)
