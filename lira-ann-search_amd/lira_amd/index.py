"""Device-resident partitioned index: the MI355X replacement for search.cpp's
``std::vector<Bucket>`` (search.cpp:273-276, 366-404) and for the per-bucket
faiss flat indexes of ``create_flat_indexes`` (utils.py:407-422).

All compute goes through liblira_hip.so (``_lib``); PyTorch only owns device
memory and streams.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import LiraError

METRICS = {"L2": _lib.LIRA_METRIC_L2, "inner_product": _lib.LIRA_METRIC_IP}


def normalize_metric(metric: str) -> str:
    """Metric names as LIRA_smallscale.py:62-66 / search.cpp:362-364 accept them."""
    m = (metric or "L2").lower()
    if m in ("l2", "euclidean", "euclidean_distance"):
        return "L2"
    if m in ("ip", "inner_product", "dot", "dot_product"):
        return "inner_product"
    raise ValueError(f"unknown metric {metric!r}: expected 'L2' or 'inner_product'")


def _dev(t: torch.Tensor, dtype, device) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        t = torch.from_numpy(np.ascontiguousarray(t))
    return t.to(device=device, dtype=dtype).contiguous()


def build_csr(data_2_bkt: torch.Tensor, n_bkt: int):
    """Inverted lists from a (N, n_mul) bucket assignment, -1 = empty slot.

    Same semantics as search.cpp:366-385: every non-negative bucket id of row i
    pushes i; each list is sorted ascending and de-duplicated.  Runs on the
    tensor's device.  Returns (offsets int64 host numpy (n_bkt+1), ids int32
    tensor, max_replicas int).
    """
    if data_2_bkt.dim() == 1:
        data_2_bkt = data_2_bkt[:, None]
    n, n_mul = data_2_bkt.shape
    flat = data_2_bkt.reshape(-1).to(torch.int64)
    if flat.numel() and int(flat.max()) >= n_bkt:
        raise LiraError("bucket id out of range.")  # search.cpp:375-377
    rows = torch.arange(n, device=flat.device, dtype=torch.int64).repeat_interleave(n_mul)
    valid = flat >= 0
    key = torch.unique(flat[valid] * max(n, 1) + rows[valid])  # sorted (bucket, row), unique
    b = key // max(n, 1)
    ids = (key - b * max(n, 1)).to(torch.int32)
    counts = torch.bincount(b, minlength=n_bkt)
    offsets = torch.zeros(n_bkt + 1, dtype=torch.int64, device=flat.device)
    offsets[1:] = torch.cumsum(counts, 0)
    max_rep = int(torch.bincount(ids.to(torch.int64), minlength=1).max()) if ids.numel() else 1
    return offsets.cpu().numpy(), ids, max(1, max_rep)


def _scan_flags(dedup, per_partition, fma, prune, exact, split) -> int:
    return (_lib.LIRA_SCAN_DEDUP if dedup else 0) | \
        (_lib.LIRA_SCAN_PER_PARTITION if per_partition else 0) | \
        (_lib.LIRA_SCAN_FMA if fma else 0) | \
        (0 if prune else _lib.LIRA_SCAN_NO_PRUNE) | \
        (_lib.LIRA_SCAN_EXACT if exact else 0) | \
        (0 if split else _lib.LIRA_SCAN_NO_SPLIT)


def parse_stats(v, paths: int) -> dict:
    """The 8 work counters of lira_index_stats_read as a dict (include/lira_hip.h).

    Slots [1] / [3] mean chunks_nominal / blocks_dropped on the all-exact scan
    (paths == 1) and the plan filter's removed pairs / their (query, candidate)
    pairs on the screened one (paths == 2); with both paths or none they are
    summed, reported as slot1 / slot3.  Callers read the path-specific keys
    with .get(): which ones exist depends on `paths`.
    """
    out = {"chunks_computed": v[0], "blocks": v[2], "blocks_skipped": v[4], "rechecked": v[5],
           "rescans": v[6], "survivors": v[7],
           "paths": {1: "exact", 2: "screen", 3: "exact+screen"}.get(paths, "none")}
    if paths == 1:
        out.update(chunks_nominal=v[1], blocks_dropped=v[3])
    elif paths == 2:
        out.update(pairs_pruned_plan=v[1], candidates_pruned_plan=v[3])
    else:
        out.update(slot1=v[1], slot3=v[3])
    return out


class PartitionedIndex:
    """Inverted lists of fp32 vectors on one GPU, searched by the HIP scan.

    Parameters mirror search.cpp's Args (search.cpp:18-31): d, metric
    ("L2" | "inner_product").  ``options`` are per-index tuning knobs
    (include/lira_hip.h LIRA_OPT_*: keep_tiles, split, qr, ...); none changes a
    result.  ``keep_tiles=False`` drops the fp32 tile copy (2 instead of 3
    copies of the data in HBM; the all-exact scan is then unavailable).
    """

    def __init__(self, d: int, metric: str = "L2", device: int | torch.device | None = None,
                 **options):
        self.d = int(d)
        self.metric = normalize_metric(metric)
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index)
        h = ctypes.c_void_p()
        _lib.call("lira_index_create", self.device.index, self.d, METRICS[self.metric],
                  ctypes.byref(h))
        self._h = h
        for name, value in options.items():
            self.set_option(name, value)
        self.n_lists = 0
        self.ntotal = 0
        self.list_sizes = np.zeros(0, dtype=np.int64)
        self.max_replicas = 1

    # ------------------------------------------------------------- lifetime
    def close(self):
        if getattr(self, "_h", None):
            _lib.load().lira_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---------------------------------------------------------------- build
    def add_lists(self, offsets, ids: torch.Tensor, x: torch.Tensor, max_replicas: int = 1):
        """Load inverted lists: bucket b = rows ids[offsets[b]:offsets[b+1]] of x."""
        offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
        ids = _dev(ids, torch.int32, self.device)
        x = _dev(x, torch.float32, self.device)
        if x.dim() != 2 or x.shape[1] != self.d:
            raise ValueError(f"x must be (n, {self.d})")
        n_lists = offsets.shape[0] - 1
        with torch.cuda.device(self.device):
            _lib.call("lira_index_add_partitions", self._h, n_lists,
                      offsets.ctypes.data_as(ctypes.c_void_p), _lib.ptr(ids), _lib.ptr(x),
                      x.shape[0], int(max_replicas), _lib.stream_ptr())
        self.n_lists = n_lists
        self.list_sizes = np.diff(offsets)
        self.ntotal = int(offsets[-1])
        self.max_replicas = int(max_replicas)
        return self

    def build(self, data_2_bkt, x, n_lists: int):
        """search.cpp:366-404 on the device (lira_index_build): lists from the
        (N, n_mul) bucket assignment over base vectors x."""
        d2b = _dev(data_2_bkt, torch.int32, self.device)
        if d2b.dim() == 1:
            d2b = d2b[:, None]
        x = _dev(x, torch.float32, self.device)
        if x.dim() != 2 or x.shape[1] != self.d or x.shape[0] != d2b.shape[0]:
            raise ValueError(f"x must be (N, {self.d}) with N = data_2_bkt rows")
        with torch.cuda.device(self.device):
            _lib.call("lira_index_build", self._h, int(n_lists), _lib.ptr(d2b), d2b.shape[0],
                      d2b.shape[1], _lib.ptr(x), _lib.stream_ptr())
        sizes = np.empty(n_lists, dtype=np.int64)
        v = ctypes.c_int64()
        for b in range(n_lists):
            _lib.call("lira_index_list_size", self._h, b, ctypes.byref(v))
            sizes[b] = v.value
        self.n_lists = n_lists
        self.list_sizes = sizes
        self.ntotal = int(sizes.sum())
        self.max_replicas = self._info_replicas(d2b)
        return self

    def _info_replicas(self, d2b):
        # the module derived it; mirror it host-side for dedup sizing checks
        rows = torch.sort(d2b, dim=1).values
        distinct = (rows >= 0) & torch.cat([torch.ones_like(rows[:, :1], dtype=torch.bool),
                                            rows[:, 1:] != rows[:, :-1]], dim=1)
        return max(1, int(distinct.sum(1).max())) if rows.numel() else 1

    def list_ids(self, b: int) -> np.ndarray:
        """Row ids of bucket b in STORAGE order (the set of search.cpp's bucket_ids[b]).

        With option order=1 (the L2 default) a list's rows are stored by ascending
        distance to its pivot, so this is a permutation of search.cpp's sorted list;
        compare as sets.  Search results never depend on the storage order."""
        out = np.empty(int(self.list_sizes[b]), dtype=np.int32)
        with torch.cuda.device(self.device):
            _lib.call("lira_index_list_ids", self._h, int(b), out.ctypes.data_as(ctypes.c_void_p),
                      _lib.stream_ptr())
        return out

    @classmethod
    def from_assignment(cls, x_d, data_2_bkt, n_bkt: int, metric: str = "L2", device=None, **options):
        """search.cpp:366-404: lists from data_2_bkt (N, n_mul) over base vectors x_d."""
        idx = cls(x_d.shape[1], metric, device, **options)
        return idx.build(data_2_bkt, x_d, n_bkt)

    @classmethod
    def from_cluster_ids(cls, x_d, cluster_ids, metric: str = "L2", device=None, **options):
        """From LIRA's ``cluster_ids`` (list of per-bucket id lists, utils.py:327-329)."""
        sizes = np.array([len(c) for c in cluster_ids], dtype=np.int64)
        offsets = np.zeros(len(cluster_ids) + 1, dtype=np.int64)
        offsets[1:] = np.cumsum(sizes)
        flat = np.concatenate([np.asarray(c, dtype=np.int64) for c in cluster_ids]) \
            if offsets[-1] else np.zeros(0, dtype=np.int64)
        rep = int(np.bincount(flat).max()) if flat.size else 1
        idx = cls(x_d.shape[1], metric, device, **options)
        idx.add_lists(offsets, torch.from_numpy(flat.astype(np.int32)), x_d, rep)
        return idx

    # --------------------------------------------------------------- search
    def search(self, q: torch.Tensor, probe: torch.Tensor, k: int, dedup: bool = True,
               per_partition: bool = False, out=None, stream=None, fma: bool = False,
               prune: bool = True, exact: bool = False, split: bool = True, workspace=None):
        """Scan the probed lists of every query; exact top-k.

        q (nq, d) fp32, probe (nq, nprobe_max) int32 (-1 = unused slot).
        Returns (D, I, ncand) device tensors: D/I (nq, k) -- or
        (nq, nprobe_max, k) with per_partition -- and ncand (nq,) int64, the
        candidates scanned per query (search.cpp's cmp_for_query).
        Distances are search.cpp's sequential fp32 sums bit for bit; fma=True
        accumulates with fused multiply-adds instead (LIRA_SCAN_FMA: fewer
        operations, ~1e-6 relative difference, near-ties may order differently).
        By default every candidate is screened with an fp32 FMA dot product
        under a rigorous error bound and only possible top-k members are
        re-computed in search.cpp's arithmetic (same results); exact=True runs
        the all-exact scan instead (LIRA_SCAN_EXACT), prune=False additionally
        turns off its L2 early abandon (same results; for A/B).  The screen's
        dot products run as split-bf16 MFMAs (hi/lo bf16 parts, fp32
        accumulation); split=False uses the fp32 MFMA screen instead
        (LIRA_SCAN_NO_SPLIT; same results).
        workspace: a device uint8 tensor of at least workspace_size() bytes, or
        None for the handle's cached buffer of the current stream (lira_hip.h,
        "Threading and streams").
        """
        q = _dev(q, torch.float32, self.device)
        probe = _dev(probe, torch.int32, self.device)
        if probe.dim() == 1:
            probe = probe[:, None]
        nq = q.shape[0]
        if q.dim() != 2 or q.shape[1] != self.d:
            raise ValueError(f"queries must be (nq, {self.d})")
        if probe.shape[0] != nq:
            raise ValueError("probe must have one row per query")
        npm = probe.shape[1]
        shape = (nq, npm, k) if per_partition else (nq, k)
        if out is None:
            D = torch.empty(shape, dtype=torch.float32, device=self.device)
            I = torch.empty(shape, dtype=torch.int64, device=self.device)
            ncand = torch.empty(nq, dtype=torch.int64, device=self.device)
        else:
            D, I, ncand = out
        flags = _scan_flags(dedup, per_partition, fma, prune, exact, split)
        if workspace is not None and (workspace.device != self.device or workspace.dtype != torch.uint8):
            raise ValueError(f"workspace must be a uint8 tensor on {self.device}")
        with torch.cuda.device(self.device):
            _lib.call("lira_scan_topk", self._h, _lib.ptr(q), nq, _lib.ptr(probe), npm, int(k),
                      flags, _lib.ptr(D), _lib.ptr(I), _lib.ptr(ncand),
                      None if workspace is None else _lib.ptr(workspace),
                      0 if workspace is None else workspace.numel(), _lib.stream_ptr(stream))
        return D, I, ncand

    def workspace_size(self, nq: int, nprobe: int, k: int, dedup: bool = True, per_partition: bool = False,
                       fma: bool = False, prune: bool = True, exact: bool = False, split: bool = True) -> int:
        """Bytes of the caller-supplied workspace search(..., workspace=) needs for this shape."""
        sz = ctypes.c_size_t()
        _lib.call("lira_scan_workspace_size", self._h, int(nq), int(nprobe), int(k),
                  _scan_flags(dedup, per_partition, fma, prune, exact, split), ctypes.byref(sz))
        return sz.value

    def describe(self, nq: int, nprobe: int, k: int, dedup: bool = True, exact: bool = False) -> str:
        """The scan kernel a search of this shape runs (lira_scan_describe)."""
        flags = (_lib.LIRA_SCAN_DEDUP if dedup else 0) | (_lib.LIRA_SCAN_EXACT if exact else 0)
        buf = ctypes.create_string_buffer(512)
        _lib.call("lira_scan_describe", self._h, int(nq), int(nprobe), int(k), flags, buf, 512)
        return buf.value.decode()

    def check(self, stream=None):
        """Raise if the last searches hit an out-of-range probe id."""
        with torch.cuda.device(self.device):
            _lib.call("lira_index_check", self._h, _lib.stream_ptr(stream))

    def set_profiling(self, enable: bool = True):
        """Record HIP events around the scan kernels (see profile_read)."""
        _lib.call("lira_index_set_profiling", self._h, int(bool(enable)))

    def profile_read(self) -> dict:
        """Summed kernel milliseconds since the last read: plan / scan / merge."""
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int64()
        with torch.cuda.device(self.device):
            _lib.call("lira_index_profile_read", self._h, ctypes.byref(a), ctypes.byref(b),
                      ctypes.byref(c), ctypes.byref(n))
        return {"plan_ms": a.value, "scan_ms": b.value, "merge_ms": c.value, "calls": n.value}

    def set_stats(self, enable: bool = True):
        """Count scan work (16-dim chunks computed vs a full scan; see stats_read)."""
        _lib.call("lira_index_set_stats", self._h, int(bool(enable)))

    def stats_read(self) -> dict:
        """Work counters since the last read: wave-chunks computed / nominal,
        candidate blocks entered, dropped by the L2 early abandon, skipped by
        the triangle-inequality test (include/lira_hip.h)."""
        v = (ctypes.c_uint64 * 8)()
        paths = ctypes.c_int()
        with torch.cuda.device(self.device):
            _lib.call("lira_index_stats_paths", self._h, ctypes.byref(paths))
            _lib.call("lira_index_stats_read", self._h, v)
        return parse_stats(list(v), paths.value)

    def set_option(self, name: str, value) -> None:
        """Set one LIRA_OPT_* knob by name (see include/lira_hip.h)."""
        if name not in _lib.OPTIONS:
            raise ValueError(f"unknown option {name!r}: one of {sorted(_lib.OPTIONS)}")
        _lib.call("lira_index_set_option", self._h, _lib.OPTIONS[name], int(value))

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        _lib.call("lira_index_get_option", self._h, _lib.OPTIONS[name], ctypes.byref(v))
        return v.value

    @property
    def has_tiles(self) -> bool:
        """True if the fp32 tile copy (all-exact scan) is resident."""
        v = ctypes.c_int()
        _lib.call("lira_index_has_tiles", self._h, ctypes.byref(v))
        return bool(v.value)

    def memory_bytes(self) -> int:
        v = ctypes.c_int64()
        _lib.call("lira_index_memory", self._h, ctypes.byref(v))
        return v.value


# ------------------------------------------------------------------ ranking
def centroid_dist(q: torch.Tensor, centroids: torch.Tensor, scaler_mean=None, scaler_scale=None,
                  out=None, stream=None) -> torch.Tensor:
    """Exact query->centroid Euclidean distances (search.cpp:220-250), (nq, B)."""
    q = _dev(q, torch.float32, q.device if isinstance(q, torch.Tensor) and q.is_cuda else "cuda")
    dev = q.device
    c = _dev(centroids, torch.float32, dev)
    nq, d = q.shape
    nb = c.shape[0]
    if c.shape[1] != d:
        raise ValueError("centroid dim != query dim")
    m = _dev(scaler_mean, torch.float32, dev) if scaler_mean is not None else None
    s = _dev(scaler_scale, torch.float32, dev) if scaler_scale is not None else None
    if (m is None) != (s is None):
        raise ValueError("scaler_mean and scaler_scale go together")
    if m is not None and (m.numel() != nb or s.numel() != nb):
        raise LiraError("Scaler dimension mismatch.")  # search.cpp:242-244
    out = torch.empty((nq, nb), dtype=torch.float32, device=dev) if out is None else out
    with torch.cuda.device(dev):
        _lib.call("lira_centroid_dist", _lib.ptr(q), nq, _lib.ptr(c), nb, d, _lib.ptr(m),
                  _lib.ptr(s), _lib.ptr(out), _lib.stream_ptr(stream))
    return out


def centroid_gemm(q: torch.Tensor, centroids: torch.Tensor, stream=None):
    """MFMA ranking GEMM: approximate squared distances (nq, B) + error bound (nq,)."""
    dev = q.device
    c = _dev(centroids, torch.float32, dev)
    q = _dev(q, torch.float32, dev)
    nq, d = q.shape
    nb = c.shape[0]
    A = torch.empty((nq, nb), dtype=torch.float32, device=dev)
    err = torch.empty(nq, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _lib.call("lira_centroid_gemm", _lib.ptr(q), nq, _lib.ptr(c), nb, d, _lib.ptr(A),
                  _lib.ptr(err), _lib.stream_ptr(stream))
    return A, err


class RankWorkspace:
    """Pre-sized workspace for rank_nearest (keeps the call graph-capturable)."""

    def __init__(self, nq: int, nb: int, device):
        sz = ctypes.c_size_t()
        _lib.call("lira_rank_workspace_size", nq, nb, ctypes.byref(sz))
        self.buf = torch.empty(max(1, sz.value), dtype=torch.uint8, device=device)
        self.nq, self.nb = nq, nb


def rank_nearest(q: torch.Tensor, centroids: torch.Tensor, nprobe: int, out=None,
                 workspace: RankWorkspace | None = None, stream=None) -> torch.Tensor:
    """IVF probe list: the nprobe nearest centroids by the exact search.cpp
    distance (ties -> smaller bucket), via the MFMA GEMM + exact re-check."""
    dev = q.device
    c = _dev(centroids, torch.float32, dev)
    q = _dev(q, torch.float32, dev)
    nq, d = q.shape
    nb = c.shape[0]
    out = torch.empty((nq, nprobe), dtype=torch.int32, device=dev) if out is None else out
    if workspace is None or workspace.nq < nq or workspace.nb != nb:
        workspace = RankWorkspace(nq, nb, dev)
    with torch.cuda.device(dev):
        _lib.call("lira_rank_nearest", _lib.ptr(q), nq, _lib.ptr(c), nb, d, int(nprobe),
                  _lib.ptr(out), _lib.ptr(workspace.buf), workspace.buf.numel(),
                  _lib.stream_ptr(stream))
    return out


def order_probes(probe: torch.Tensor, key: torch.Tensor, stream=None) -> torch.Tensor:
    """Reorder each row of an (n, max_probe) -1 padded probe matrix IN PLACE by
    ascending key[i, b] (ties -> smaller b, -1 last): lira_order_probes.  Same
    probe sets, so the same scan results; with key = query -> centroid distance
    the scan sees each query's nearest probed partition first (its seed and
    nearest-probe group).  Returns probe."""
    if probe.dtype != torch.int32 or not probe.is_contiguous():
        raise ValueError("probe must be a contiguous int32 tensor")
    k = _dev(key, torch.float32, probe.device)
    n, mp = probe.shape
    if k.shape[0] != n:
        raise ValueError("key rows != probe rows")
    with torch.cuda.device(probe.device):
        _lib.call("lira_order_probes", _lib.ptr(probe), n, mp, _lib.ptr(k), k.shape[1], _lib.stream_ptr(stream))
    return probe


def select_probes(scores: torch.Tensor, mode: str, max_probe: int, threshold: float = 0.0,
                  stream=None, by_score: bool = False):
    """Probe lists from an (n, B) score matrix.

    mode "nearest": max_probe smallest; "ge": score >= threshold with argmax
    fallback (search.cpp:447-466); "gt": score > threshold (LIRA_smallscale.py:206).
    by_score: the threshold set in descending score order (LIRA_PROBE_BY_SCORE).
    Returns (probe (n, max_probe) int32 -1 padded, nprobe (n,) int32).
    """
    modes = {"nearest": _lib.LIRA_PROBE_NEAREST, "ge": _lib.LIRA_PROBE_THRESHOLD_GE,
             "gt": _lib.LIRA_PROBE_THRESHOLD_GT}
    s = _dev(scores, torch.float32, scores.device)
    n, nb = s.shape
    probe = torch.empty((n, max_probe), dtype=torch.int32, device=s.device)
    cnt = torch.empty(n, dtype=torch.int32, device=s.device)
    m = modes[mode] | (_lib.LIRA_PROBE_BY_SCORE if by_score else 0)
    with torch.cuda.device(s.device):
        _lib.call("lira_select_probes", _lib.ptr(s), n, nb, m, float(threshold),
                  int(max_probe), _lib.ptr(probe), _lib.ptr(cnt), _lib.stream_ptr(stream))
    return probe, cnt
