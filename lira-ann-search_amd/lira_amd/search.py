"""End-to-end artifact search on the GPU: the search.cpp pipeline
(search.cpp:278-558) with the hot path on the HIP module.

Per query batch (search.cpp:421-514, batched instead of one query at a time):
    exact query->centroid distances + standardisation   lira_centroid_dist
    probing MLP scores                                    PyTorch-ROCm (probing.py)
    probe buckets with score >= thr, argmax fallback      lira_select_probes
    scan the probed buckets, exact top-k                  lira_scan_topk
then recall@k against the ground truth (search.cpp:519-528) and QPS =
queries / wall time of the pipeline (search.cpp:540), per threshold of the
sweep (search.cpp:413; integer steps instead of float accumulation).

CLI, with search.cpp's flags (search.cpp:18-82):
    python -m lira_amd.search --dataset sift --data_path /data/vector_datasets \
        --artifacts_dir DIR --prefix NAME --k 10 --metric L2 [--t_min --t_max --t_step]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

from .index import PartitionedIndex, build_csr, centroid_dist, normalize_metric, select_probes
from .io import load_artifacts, read_fvecs, read_ivecs
from .probing import probe_scores


def recall_at_k(I: np.ndarray, gt: np.ndarray, k: int) -> np.ndarray:
    """search.cpp:519-528: |gt[:k] intersect found| / k for each query."""
    out = np.empty(I.shape[0])
    for i in range(I.shape[0]):
        found = set(int(v) for v in I[i] if v >= 0)
        out[i] = sum(int(g) in found for g in gt[i, :k]) / k
    return out


def thresholds(t_min: float, t_max: float, t_step: float, cpp_exact: bool = True) -> np.ndarray:
    """The sweep of search.cpp:413.

    cpp_exact (default) reproduces the reference's fp32 accumulation
    `for (float thr = t_min; thr <= t_max + 1e-6f; thr += t_step)` value for
    value, so a score equal to a threshold probes exactly as search.cpp does;
    otherwise thresholds are t_min + i * t_step in float64, rounded once.
    """
    if not cpp_exact:
        n = int(np.floor((t_max - t_min) / t_step + 1e-6)) + 1
        return (t_min + t_step * np.arange(max(0, n))).astype(np.float32)
    out = []
    thr, lim, step = np.float32(t_min), np.float32(np.float32(t_max) + np.float32(1e-6)), np.float32(t_step)
    while thr <= lim and len(out) < 1_000_000:
        out.append(thr)
        thr = np.float32(thr + step)
    return np.array(out, dtype=np.float32)


class SearchEngine:
    """search.cpp's loaded state: inverted lists, centroids, scaler, model."""

    def __init__(self, artifacts, metric: str = "L2", device: int = 0, dedup: bool = False):
        if isinstance(artifacts, str):
            artifacts = load_artifacts(artifacts, device=f"cuda:{device}")
        self.device = torch.device("cuda", device)
        self.metric = normalize_metric(metric)
        dev = self.device
        self.centroids = torch.from_numpy(artifacts["centroids"]).to(dev)
        self.n_bkt, self.d = self.centroids.shape
        self.mean = torch.from_numpy(artifacts["scaler_mean"]).to(dev)
        self.scale = torch.from_numpy(artifacts["scaler_scale"]).to(dev)
        self.model = artifacts["model"].to(dev).eval()
        x = torch.from_numpy(np.ascontiguousarray(artifacts["x_d"])).to(dev)
        d2b = torch.from_numpy(np.ascontiguousarray(artifacts["data_2_bkt"])).to(dev)
        offsets, ids, rep = build_csr(d2b, self.n_bkt)
        self.index = PartitionedIndex(self.d, self.metric, device)
        self.index.add_lists(offsets, ids, x, rep)
        del x
        self.dedup = dedup  # search.cpp keeps replicated gids twice (Appendix A)
        self._pipe, self._pipe_key = None, None

    def scores(self, q: torch.Tensor) -> torch.Tensor:
        dist = centroid_dist(q, self.centroids, self.mean, self.scale)
        return probe_scores(self.model, dist, q)

    def pipeline(self, nq: int, k: int) -> "ProbePipeline":
        """The ProbePipeline of a batch shape (built once per (nq, k); the
        threshold is an argument of each run)."""
        key = (int(nq), int(k))
        if self._pipe is None or self._pipe_key != key:
            self._pipe = ProbePipeline(self.index, self.centroids, self.mean, self.scale, self.model,
                                       int(nq), int(k), 0.5, max_probe=self.n_bkt, dedup=self.dedup)
            self._pipe_key = key
        return self._pipe

    def search(self, q, threshold: float, k: int, scores: torch.Tensor | None = None):
        """One threshold: returns fresh (D, I, nprobe, ncand) device tensors.

        Without precomputed ``scores`` this runs the ProbePipeline of the
        batch shape (distances + standardise in one kernel, MLP, select, scan
        on preallocated buffers) and returns copies of its outputs, so a later
        search never overwrites them."""
        q = q if isinstance(q, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(q))
        q = q.to(self.device, torch.float32).contiguous()
        if scores is None:
            p = self.pipeline(q.shape[0], k)
            p.q.copy_(q)
            p.run(threshold)
            return p.D.clone(), p.I.clone(), p.nprobe.clone(), p.ncand.clone()
        probe, nprobe = select_probes(scores, "ge", self.n_bkt, threshold)
        D, I, ncand = self.index.search(q, probe, k, dedup=self.dedup)
        return D, I, nprobe, ncand

    def sweep(self, q, gt, k: int, t_min=0.02, t_max=0.80, t_step=0.02, verbose=True):
        """search.cpp:413-548 for a query set; one row per threshold."""
        qt = torch.from_numpy(np.ascontiguousarray(q)).to(self.device)
        k = min(k, gt.shape[1])  # search.cpp:357-360 clamps k to the gt width
        self.pipeline(qt.shape[0], k)  # (buffers allocated outside the timed region)
        rows = []
        for thr in thresholds(t_min, t_max, t_step):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D, I, nprobe, ncand = self.search(qt, float(thr), k)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            rec = recall_at_k(I.cpu().numpy(), gt, k)
            row = {"threshold": float(thr), "avg_recall": float(rec.mean()),
                   "avg_nprobe": float(nprobe.float().mean()), "avg_cmp": float(ncand.double().mean()),
                   "avg_time": dt / len(q), "qps": len(q) / dt}
            rows.append(row)
            if verbose:
                print(f"=== Threshold = {thr:g} ===\nThreshold    : {thr:g}\n"
                      f"avg_recall   : {row['avg_recall']:g}\navg_nprobe   : {row['avg_nprobe']:g}\n"
                      f"avg_cmp      : {row['avg_cmp']:g}\navg_time(q)  : {row['avg_time']:g} s\n"
                      f"QPS          : {row['qps']:g} q/s\n----------------------------------------")
        return rows


class ProbePipeline:
    """search.cpp's per-query pipeline (search.cpp:424-514) for a fixed batch
    shape, on preallocated device buffers so the whole chain can be captured in
    one HIP graph (no allocation, no host synchronisation inside):

        exact query->centroid distances + standardise   lira_centroid_dist (one kernel)
        probing MLP                                      PyTorch-ROCm (hipBLASLt)
        score >= thr, argmax fallback                    lira_select_probes
        the same set, nearest centroid first             lira_order_probes (raw distance
                                                         = standardised * scale + mean)
        scan + exact top-k                               lira_scan_topk

    The probe ORDER never changes a result (lira_scan_topk's output is order
    independent); it sets the scan's speed: slot 0 seeds each query's starting
    bound and forms the nearest-probe group, so the nearest probed partition
    belongs there (a score-ordered selection put an arbitrary one of the ~8
    near-equal-score partitions first: SIFT1M mixture screen 0.57 -> 0.33 ms).

    ``max_probe`` caps the probe list per query (search.cpp has no cap: pass
    n_bkt for its exact semantics).
    """

    def __init__(self, index: PartitionedIndex, centroids, scaler_mean, scaler_scale, model, nq: int, k: int,
                 threshold: float, max_probe: int | None = None, dedup: bool = True,
                 expect_probes: int | None = None):
        dev = index.device
        self.index, self.model, self.k, self.thr, self.dedup = index, model, int(k), float(threshold), dedup
        self.C = torch.as_tensor(centroids, dtype=torch.float32).to(dev).contiguous()
        self.mean = torch.as_tensor(scaler_mean, dtype=torch.float32).to(dev).contiguous()
        self.scale = torch.as_tensor(scaler_scale, dtype=torch.float32).to(dev).contiguous()
        nb = self.C.shape[0]
        self.max_probe = int(max_probe or nb)
        self.q = torch.zeros((nq, index.d), dtype=torch.float32, device=dev)
        self.dist = torch.empty((nq, nb), dtype=torch.float32, device=dev)
        self.probe = torch.empty((nq, self.max_probe), dtype=torch.int32, device=dev)
        self.nprobe = torch.empty(nq, dtype=torch.int32, device=dev)
        self.D = torch.empty((nq, k), dtype=torch.float32, device=dev)
        self.I = torch.empty((nq, k), dtype=torch.int64, device=dev)
        self.ncand = torch.empty(nq, dtype=torch.int64, device=dev)
        # the model's output lands in an fp32 buffer of its own (any output dtype or
        # layout is converted by the copy; keeps the chain graph-capturable)
        self.scores = torch.empty((nq, nb), dtype=torch.float32, device=dev)
        self.raw = torch.empty((nq, nb), dtype=torch.float32, device=dev)  # unstandardised distances (order key)
        self.graph = None
        # search.cpp's set (>= thr, argmax fallback); ordered by descending score
        # where the list fits (same results, faster scan: most probable partition first)
        from . import _lib
        self.mode = _lib.LIRA_PROBE_THRESHOLD_GE | (_lib.LIRA_PROBE_BY_SCORE if self.max_probe <= 256 else 0)
        # a performance hint for the scan's work split (LIRA_OPT_PROBES_HINT), applied
        # around this pipeline's own scans only
        self.expect_probes = int(expect_probes or 0)

    @torch.no_grad()
    def run(self, threshold: float | None = None):
        """One pass over self.q (stream-ordered, asynchronous), at `threshold`
        (default: the pipeline's own).  A new threshold drops a captured graph:
        the graph holds lira_select_probes' threshold argument of capture time."""
        if threshold is not None and float(threshold) != self.thr:
            self.thr = float(threshold)
            self.graph = None
        centroid_dist(self.q, self.C, self.mean, self.scale, out=self.dist)
        self.scores.copy_(self.model(self.dist, self.q))
        self._select_scan()

    def _select_scan(self):
        from . import _lib
        with torch.cuda.device(self.q.device):
            _lib.call("lira_select_probes", _lib.ptr(self.scores), self.q.shape[0], self.C.shape[0],
                      self.mode, self.thr, self.max_probe, _lib.ptr(self.probe), _lib.ptr(self.nprobe),
                      _lib.stream_ptr())
            if self.max_probe <= 256:  # nearest probed partition first (speed only)
                torch.addcmul(self.mean, self.dist, self.scale, out=self.raw)
                _lib.call("lira_order_probes", _lib.ptr(self.probe), self.q.shape[0], self.max_probe,
                          _lib.ptr(self.raw), self.C.shape[0], _lib.stream_ptr())
        old = self.index.get_option("probes_hint") if self.expect_probes else None
        if self.expect_probes:
            self.index.set_option("probes_hint", self.expect_probes)
        try:
            self.index.search(self.q, self.probe, self.k, dedup=self.dedup, out=(self.D, self.I, self.ncand))
        finally:
            if old is not None:
                self.index.set_option("probes_hint", old)

    def capture(self):
        """Record run() into a HIP graph (after one eager warm-up run, so the
        scan's cached workspace is already sized)."""
        s = torch.cuda.Stream(device=self.q.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.run()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.run()
        return self

    def replay(self):
        if self.graph is None:
            raise RuntimeError("ProbePipeline.replay: no captured graph (capture() first; run() at a new "
                               "threshold drops the graph, whose selection threshold is fixed at capture)")
        self.graph.replay()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="LIRA end-to-end search on MI355X (search.cpp flags)")
    ap.add_argument("--dataset", required=True)
    ap.add_argument("--data_path", default="/data/vector_datasets")
    ap.add_argument("--artifacts_dir", default=".")
    ap.add_argument("--prefix", required=True)
    ap.add_argument("--metric", default="L2")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--num_threads", type=int, default=32, help="accepted for compatibility")
    ap.add_argument("--t_min", type=float, default=0.02)
    ap.add_argument("--t_max", type=float, default=0.80)
    ap.add_argument("--t_step", type=float, default=0.02)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--dedup", action="store_true", help="keep each gid once (search.cpp does not)")
    a = ap.parse_args(argv)
    try:
        prefix = os.path.join(a.artifacts_dir, a.prefix)
        eng = SearchEngine(prefix, a.metric, a.device, a.dedup)
        ddir = os.path.join(a.data_path, a.dataset)
        q = np.ascontiguousarray(read_fvecs(os.path.join(ddir, f"{a.dataset}_query.fvecs")))
        gt = np.ascontiguousarray(read_ivecs(os.path.join(ddir, f"{a.dataset}_groundtruth.ivecs")))
        if q.shape[1] != eng.d:
            raise ValueError("query dim != base dim.")
        if gt.shape[0] != q.shape[0]:
            raise ValueError("groundtruth and queries count mismatch.")
        print(f"Dataset      : {a.dataset}\nPrefix       : {prefix}\nMetric       : {a.metric}\nK            : {a.k}")
        eng.sweep(q, gt, a.k, a.t_min, a.t_max, a.t_step)
        print("Done.")
    except Exception as e:  # search.cpp:552-555
        print(f"[Error] {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
