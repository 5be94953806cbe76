"""numpy front-end of the CPU oracle (oracle/lira_oracle.c).

TEST INFRASTRUCTURE ONLY -- the parity checker for the HIP path and the
cpu_baseline leg of bench.py.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline import this module; the product (lira_amd) never does.

Each wrapper cites the reference lines its C function restates; see the header
of lira_oracle.c.  Also exposes the reference's OWN compiled functions
(oracle/_ref/libref_search.so, built from /root/reference/search.cpp by
`make -C oracle ref`) when that library is present, to pin the restatement.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liblira_oracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libref_search.so")

L2, IP = 0, 1
_P = ctypes.c_void_p
_I64 = ctypes.c_int64

_lib = None
_ref = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_l2_sq.restype = ctypes.c_float
        L.oracle_l2_sq.argtypes = [_P, _P, _I64]
        L.oracle_ip.restype = ctypes.c_float
        L.oracle_ip.argtypes = [_P, _P, _I64]
        L.oracle_centroid_dist.argtypes = [_P, _I64, _P, _I64, _I64, _P]
        L.oracle_standardize.argtypes = [_P, _I64, _I64, _P, _P]
        L.oracle_build_csr.restype = _I64
        L.oracle_build_csr.argtypes = [_P, _I64, _I64, _I64, _P, _P]
        L.oracle_probe_threshold.argtypes = [_P, _I64, _I64, ctypes.c_float, ctypes.c_int, _P, _P]
        L.oracle_probe_nearest.argtypes = [_P, _I64, _I64, _I64, _P]
        L.oracle_scan_topk.argtypes = [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64, ctypes.c_int,
                                       ctypes.c_int, _P, _P, _P]
        L.oracle_scan_per_partition.argtypes = [_P, _I64, _I64, _P, _P, _P, _P, _I64, _I64,
                                                ctypes.c_int, _P, _P]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_num_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def ref() -> ctypes.CDLL | None:
    """The reference's own search.cpp functions, or None when not built here."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB):
        R = ctypes.CDLL(REF_LIB, mode=os.RTLD_LAZY)  # cnpy::npy_load stays unbound
        for f in (R.ref_l2_sq, R.ref_ip):
            f.restype = ctypes.c_float
            f.argtypes = [_P, _P, ctypes.c_long]
        R.ref_centroid_dist.argtypes = [_P, _P, ctypes.c_long, ctypes.c_long, _P, _P, _P]
        _ref = R
    return _ref


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _p(a):
    return a.ctypes.data_as(_P) if a is not None else None


def set_threads(n: int) -> None:
    lib().oracle_set_num_threads(int(n))


def num_threads() -> int:
    return lib().oracle_num_threads()


def l2_sq(a, b) -> np.float32:
    """search.cpp:253-260"""
    a, b = _c(a, np.float32), _c(b, np.float32)
    return np.float32(lib().oracle_l2_sq(_p(a), _p(b), a.shape[0]))


def ip(a, b) -> np.float32:
    """search.cpp:263-269"""
    a, b = _c(a, np.float32), _c(b, np.float32)
    return np.float32(lib().oracle_ip(_p(a), _p(b), a.shape[0]))


def centroid_dist(q, cent, mean=None, scale=None) -> np.ndarray:
    """search.cpp:220-235 (+ :238-250 when mean/scale given), batched."""
    q, cent = _c(q, np.float32), _c(cent, np.float32)
    out = np.empty((q.shape[0], cent.shape[0]), dtype=np.float32)
    lib().oracle_centroid_dist(_p(q), q.shape[0], _p(cent), cent.shape[0], q.shape[1], _p(out))
    if mean is not None:
        m, s = _c(mean, np.float32), _c(scale, np.float32)
        lib().oracle_standardize(_p(out), out.shape[0], out.shape[1], _p(m), _p(s))
    return out


def build_csr(data_2_bkt, n_bkt):
    """search.cpp:366-385 -> (offsets int64 (n_bkt+1), ids int32)."""
    d2b = _c(data_2_bkt, np.int32)
    if d2b.ndim == 1:
        d2b = d2b[:, None]
    offsets = np.zeros(n_bkt + 1, dtype=np.int64)
    ids = np.empty(max(1, d2b.size), dtype=np.int32)
    n = lib().oracle_build_csr(_p(d2b), d2b.shape[0], d2b.shape[1], n_bkt, _p(offsets), _p(ids))
    if n < 0:
        raise RuntimeError("bucket id out of range.")
    return offsets, ids[:n].copy()


def gather_lists(x, offsets, ids):
    """search.cpp:387-403: contiguous per-bucket copies of x rows."""
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32)[ids])


def probe_threshold(scores, thr, strict=False):
    """search.cpp:447-466 (strict=False) / LIRA_smallscale.py:206 (strict=True)."""
    s = _c(scores, np.float32)
    out = np.empty(s.shape, dtype=np.int32)
    cnt = np.empty(s.shape[0], dtype=np.int32)
    lib().oracle_probe_threshold(_p(s), s.shape[0], s.shape[1], float(thr), int(strict), _p(out), _p(cnt))
    return out, cnt


def probe_nearest(dist, nprobe):
    d = _c(dist, np.float32)
    out = np.empty((d.shape[0], nprobe), dtype=np.int32)
    lib().oracle_probe_nearest(_p(d), d.shape[0], d.shape[1], nprobe, _p(out))
    return out


def scan_topk(q, offsets, ids, vecs, probe, k, metric=L2, dedup=0):
    """search.cpp:471-514 in canonical (score, gid) order.  dedup: 0 off, r>0 on
    (r = max buckets per gid).  Returns (D, I, ncand)."""
    q = _c(q, np.float32)
    offsets, ids, vecs = _c(offsets, np.int64), _c(ids, np.int32), _c(vecs, np.float32)
    probe = _c(probe, np.int32)
    if probe.ndim == 1:
        probe = probe[:, None]
    nq, d = q.shape
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    nc = np.empty(nq, dtype=np.int64)
    lib().oracle_scan_topk(_p(q), nq, d, _p(offsets), _p(ids), _p(vecs), _p(probe),
                           probe.shape[1], k, metric, int(dedup), _p(D), _p(I), _p(nc))
    return D, I, nc


def scan_topk_sampled(q, probe, list_ids, gather, k, metric=L2, dedup=0, threads=8):
    """scan_topk of each query over its own probed lists only (a per-query
    sub-CSR), for indexes too large to copy to the host whole.

    q (n, d) and probe (n, nprobe) host arrays; list_ids(b) -> the bucket's
    ids (int32, list order); gather(ids) -> their vectors (host fp32 array).
    Inputs are prepared one query at a time in the calling thread (gather is
    called per bucket, so the caller's device memory holds one list at a
    time) and scanned by `threads` worker threads (the C call releases the
    GIL), at most 2 x threads queries in flight.  Returns (D, I)."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    q = _c(q, np.float32)
    probe = np.asarray(probe)
    gate = threading.Semaphore(2 * max(1, threads))

    def run(args):
        try:
            qi, off, ids, vecs, sub = args
            D, I, _ = scan_topk(qi, off, ids, vecs, sub, k, metric, dedup)
            return D[0], I[0]
        finally:
            gate.release()

    futs = []
    with ThreadPoolExecutor(max(1, threads)) as ex:
        for i in range(q.shape[0]):
            bs = [int(b) for b in probe[i] if b >= 0]
            ls = [np.asarray(list_ids(b), dtype=np.int32) for b in bs]
            off = np.zeros(len(ls) + 1, dtype=np.int64)
            off[1:] = np.cumsum([len(l) for l in ls])
            ids = np.concatenate(ls) if ls else np.zeros(0, np.int32)
            vecs = np.concatenate([gather(l) for l in ls]) if ls else np.zeros((0, q.shape[1]), np.float32)
            gate.acquire()
            futs.append(ex.submit(run, (q[i:i + 1], off, ids, vecs, np.arange(len(ls), dtype=np.int32)[None, :])))
        res = [f.result() for f in futs]
    if not res:
        return np.zeros((0, k), np.float32), np.zeros((0, k), np.int64)
    return np.stack([r[0] for r in res]), np.stack([r[1] for r in res])


def scan_per_partition(q, offsets, ids, vecs, probe, k, metric=L2):
    """LIRA_smallscale.py:145-174: k best per probed bucket, (nq, nprobe, k)."""
    q = _c(q, np.float32)
    offsets, ids, vecs = _c(offsets, np.int64), _c(ids, np.int32), _c(vecs, np.float32)
    probe = _c(probe, np.int32)
    nq, d = q.shape
    npm = probe.shape[1]
    D = np.empty((nq, npm, k), dtype=np.float32)
    I = np.empty((nq, npm, k), dtype=np.int64)
    lib().oracle_scan_per_partition(_p(q), nq, d, _p(offsets), _p(ids), _p(vecs), _p(probe), npm,
                                    k, metric, _p(D), _p(I))
    return D, I


# -------------------------------------------------- pure numpy restatements
def l2_sq_np(a, b) -> np.float32:
    """search.cpp:253-260 as an explicit fp32 loop (small cases only)."""
    acc = np.float32(0.0)
    for x, y in zip(np.asarray(a, np.float32), np.asarray(b, np.float32)):
        df = np.float32(x - y)
        acc = np.float32(acc + np.float32(df * df))
    return acc


def recall_at_k(found_ids, gt_ids, k):
    """search.cpp:519-528: |gt[:k] ∩ found| / k per query."""
    found_ids = np.asarray(found_ids)
    gt_ids = np.asarray(gt_ids)
    out = np.empty(found_ids.shape[0])
    for i in range(found_ids.shape[0]):
        s = set(int(v) for v in found_ids[i] if v >= 0)
        out[i] = sum(int(g) in s for g in gt_ids[i, :k]) / k
    return out


def merge_shards(Dp, Ip, ip, dedup, k):
    """lira_merge_shards restated (test infrastructure): the k smallest keys of the
    union of P per-shard (nq, k) top-k lists in search.cpp:495-514's order --
    ascending (score, gid), score = D for L2 and -D for IP -- equal keys (a row
    reached through buckets of two shards) kept once with dedup.  Pads: I = -1."""
    Dp, Ip = np.asarray(Dp), np.asarray(Ip)
    P, nq = Dp.shape[0], Dp.shape[1]
    outD = np.full((nq, k), -np.inf if ip else np.inf, dtype=np.float32)
    outI = np.full((nq, k), -1, dtype=np.int64)
    for qi in range(nq):
        keys = sorted((float(-Dp[p, qi, j]) if ip else float(Dp[p, qi, j]), int(Ip[p, qi, j]), Dp[p, qi, j])
                      for p in range(P) for j in range(Dp.shape[2]) if Ip[p, qi, j] >= 0)
        out, last = 0, None
        for sc, gid, dv in keys:
            if out == k:
                break
            if dedup and last == (sc, gid):
                continue
            outD[qi, out], outI[qi, out] = dv, gid
            out += 1
            last = (sc, gid)
    return outD, outI
