"""Benchmark of LIRA's query-time hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config sift1m] [--data mixture|latent]
                    [--scaling weak|strong] [--opt name=value ...]

One step = one pass of the hot path over one batch of synthetic queries on
every rank: MFMA ranking GEMM + exact nprobe boundary re-check
(lira_rank_nearest) -> batched scan + exact top-k (lira_scan_topk) -> for
N > 1 an RCCL all-gather of the per-rank top-k (every rank holds a full index
replica).  Inputs are resident in HBM before the timed region.
Rank 0 prints ONE JSON line (the bench contract).

Scaling: ``weak`` (default) gives every rank its own batch of --nq queries;
``strong`` splits one batch of --nq queries over the ranks (lira_amd.distributed
.shard_bounds), so at N = 1 it is the same workload and at N = 8 each rank scans
nq/8 queries.  value = queries of all ranks / max-over-ranks time.

Partition shards (--shard partitions): rank r builds only the lists of the
buckets partition_owners gives it (B/N of the data), all ranks rank and scan
the same batch, and a step ends with the all-gather of the N per-rank top-k
and their k-way merge on the device (lira_merge_shards): value = the batch's
queries / max-over-ranks time (strong scaling).

Multi-GPU: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the
environment starts N ranks itself (a child `python -m torch.distributed.run
--nproc-per-node N ... bench.py` process; this parent never touches the GPU and
exits with the child's status).  Under torch.distributed.run (the driver's
form) it runs as one of the ranks.  Every N > 1 line carries both figures:
`value` for --scaling (weak by default) and an `other_scaling` sub-record for
the other mode on the same index, plus `ranks_seen` (the world size the
process group reported and each rank's device).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lira-ann-search_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# peaks (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0          # HBM3E spec
L2LDS_PEAK_GBS = 18800.0       # LDS-DMA gather into LDS from the XCD L2, chip-wide (upper end, measured)
L2_PEAK_GBS = 34500.0          # L2 read bandwidth, chip-wide (MI355X_MICROARCH.md, L2 per XCD)
MFMA_F32_PEAK_TFLOPS = 157.3   # v_mfma_f32_*_f32 dense = fp32 vector peak
MFMA_BF16_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA, 16 x the f32 rate
VALU_F32_PEAK_TOPS = 78.64     # non-FMA fp32 lane ops/s (157.3 TFLOP/s counts an FMA as 2)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="sift1m", choices=["sift1m", "gist1m", "deep10m", "bigann100m"])
    ap.add_argument("--nq", type=int, default=None, help="queries per rank (weak) / per job (strong) per step")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--recall-sample", type=int, default=100)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--fma", action="store_true",
                    help="LIRA_SCAN_FMA accumulation (tolerance variant, not the reference's rounding)")
    ap.add_argument("--data", default="mixture", choices=["latent", "mixture", "uniform"],
                    help="synthetic distribution (lira_amd/synthetic.py): mixture = SURVEY 8(d)'s "
                         "Gaussian mixture (default); latent = low intrinsic dimension + k-means "
                         "partitions, recall near the metric's 0.95 point like real SIFT1M")
    ap.add_argument("--contrast", default="auto", choices=["auto", "none"],
                    help="auto: at N=1 on sift1m/gist1m also time the other distribution "
                         "(reported as contrast_data, outside the headline's timed region)")
    ap.add_argument("--opt", action="append", default=[],
                    help="index option name=value (include/lira_hip.h LIRA_OPT_*), repeatable")
    ap.add_argument("--sweep", action="append", default=[],
                    help="name=v1,v2,...: after the timed run, re-time the step with each value of an index "
                         "option (include/lira_hip.h LIRA_OPT_*) on the same index and batch (rank 0, N=1)")
    ap.add_argument("--no-exact", action="store_true", help="skip the all-exact kernel comparison")
    ap.add_argument("--graph", type=int, default=1,
                    help="1 (default): the step's rank + search launches replayed as one captured HIP graph "
                         "(hipGraph via torch.cuda.CUDAGraph; collectives stay outside); 0: launched one by one")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the MLP-probed pipeline timing")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--shard", default="queries", choices=["queries", "partitions"],
                    help="queries (default): every rank holds the whole index and scans its own queries; "
                         "partitions: rank r holds the lists of its buckets only (lira_amd.distributed."
                         "partition_owners), every rank scans the whole batch against them, and the ranks' "
                         "top-k are all-gathered and merged on the device (lira_merge_shards) -- SURVEY 8(e)'s "
                         "mode for BIGANN's memory; strong scaling by construction")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def oracle_sample(oracle, idx, x, q, probe, rows, k, metric, lists, threads=8):
    """search.cpp's scan (oracle/lira_oracle.c) of each sampled query over its
    own probed lists (a per-query sub-CSR: works for an index larger than host
    memory).  Returns (D, I) of the sampled rows."""
    met = oracle.IP if metric == "inner_product" else oracle.L2

    def gather(ids):
        return x[torch.from_numpy(ids).to(x.device).long()].cpu().numpy()

    return oracle.scan_topk_sampled(q.cpu().numpy()[rows], probe.cpu().numpy()[rows], lists, gather, k, met,
                                    idx.max_replicas, threads)


def blas_scan_topk(qs, off, ids, vecs, ps, k, ip):
    """CPU approximation of faiss IndexFlatL2/IP.search's BLAS path
    (LIRA_smallscale.py:168 calls inner_index.search per bucket): for every
    probed list, the queries that probe it in one block -> one sgemm
    (torch CPU, all threads), ||q||^2 - 2 q.x + ||x||^2 (norms computed per
    search, as faiss' exhaustive_L2sqr_blas does), top-k per (query, list), then
    top-k over each query's nprobe x k candidates with replicas de-duplicated
    (a row in two probed lists counts once, at its better score, as the GPU's
    LIRA_SCAN_DEDUP output does).  Not bit-exact with search.cpp's sequential
    sum; a baseline, not the oracle."""
    n, P = ps.shape
    worst = -np.inf if ip else np.inf
    cD = torch.full((n * P, k), worst, dtype=torch.float32)
    cI = torch.full((n * P, k), -1, dtype=torch.int64)
    Q = torch.from_numpy(np.ascontiguousarray(qs))
    qn = (Q * Q).sum(1)
    flat = ps.ravel()
    order = np.argsort(flat, kind="stable")
    fs = flat[order]
    cut = np.flatnonzero(np.diff(fs)) + 1
    for grp in np.split(order, cut):
        b = int(flat[grp[0]])
        if b < 0 or off[b + 1] == off[b]:
            continue
        lo, hi = int(off[b]), int(off[b + 1])
        X = torch.from_numpy(vecs[lo:hi])
        qi = torch.from_numpy(grp // P)
        G = Q[qi] @ X.T
        if ip:
            v, j = torch.topk(G, min(k, hi - lo), dim=1)
        else:
            G.mul_(-2).add_(qn[qi, None]).add_((X * X).sum(1)[None, :])
            v, j = torch.topk(G, min(k, hi - lo), dim=1, largest=False)
        rows = torch.from_numpy(grp)
        cD[rows, :v.shape[1]] = v
        cI[rows, :v.shape[1]] = torch.from_numpy(ids[lo:hi])[j.reshape(-1)].reshape(j.shape).long()
    cD, cI = cD.view(n, P * k), cI.view(n, P * k)
    # de-duplicate ids: group each row by id (stable sorts: by score, then by id),
    # keep the best score of each id, push the others past every real score
    o1 = torch.sort(cD, dim=1, descending=ip, stable=True).indices
    cD, cI = torch.gather(cD, 1, o1), torch.gather(cI, 1, o1)
    o2 = torch.sort(cI, dim=1, stable=True).indices
    cD, cI = torch.gather(cD, 1, o2), torch.gather(cI, 1, o2)
    dup = torch.zeros_like(cI, dtype=torch.bool)
    dup[:, 1:] = (cI[:, 1:] == cI[:, :-1]) & (cI[:, 1:] >= 0)
    cD = cD.masked_fill(dup, worst)
    cI = cI.masked_fill(dup, -1)
    v, j = torch.topk(cD, k, dim=1, largest=ip)
    return v.numpy(), torch.gather(cI, 1, j).numpy()


def time_blas(qs, ps, host, k, ip, threads, budget_s=10.0):
    """Times blas_scan_topk on a bounded prefix of the batch (pilot of 64
    queries scaled to ~budget_s seconds).  Returns (n, seconds, D, I)."""
    torch.set_num_threads(threads)
    pilot = min(64, len(qs))
    tp = time.perf_counter()
    blas_scan_topk(qs[:pilot], *host, ps[:pilot], k, ip)
    per_q = max(time.perf_counter() - tp, 1e-9) / pilot
    n = int(min(len(qs), max(pilot, budget_s / per_q)))
    tc = time.perf_counter()
    D, I = blas_scan_topk(qs[:n], *host, ps[:n], k, ip)
    return n, time.perf_counter() - tc, D, I


def parse_opts(items, config):
    opts = {}
    if config == "bigann100m":
        opts["keep_tiles"] = 0  # n_mul = 2: 2 copies (row-major + split-bf16) fit 288 GB, 3 do not
    for it in items:
        name, _, v = it.partition("=")
        opts[name.strip()] = int(v)
    return opts


def time_batch(args, index, q, centres, nprobe, k, world, dist, gdev, nq_total, scaling):
    """Time args.steps steps of the hot path on this rank's query slice q
    (rank_nearest -> scan + top-k, as one HIP graph unless --graph 0, then for
    N > 1 the all-gather of the per-rank top-k), barrier + synchronize on both
    sides, max over ranks.  Returns (elapsed s, D, I, ncand, probe, local_step,
    graph, verified): `verified` checks once, after the timed loop, that every
    rank's gathered copy of this rank's rows equals its own result (None at N = 1)."""
    from lira_amd import RankWorkspace, rank_nearest
    from lira_amd.distributed import all_gather_rows, shard_bounds
    dev = q.device
    nq = q.shape[0]
    B = centres.shape[0]
    ws = RankWorkspace(max(1, nq), B, dev)
    probe = torch.empty((nq, nprobe), dtype=torch.int32, device=dev)
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    ncand = torch.empty(nq, dtype=torch.int64, device=dev)

    def local_step():
        rank_nearest(q, centres, nprobe, out=probe, workspace=ws)
        index.search(q, probe, k, dedup=True, out=(D, I, ncand), fma=args.fma)

    # the step's ~10 launches as one HIP graph: no per-launch host overhead or
    # gaps between kernels (the library's calls are capture-safe: workspaces
    # are allocated by the warm-up calls, no host syncs on the search path)
    graph = None
    if args.graph:
        for _ in range(2):
            local_step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            local_step()
        torch.cuda.synchronize()

    def gather():
        if scaling == "strong":
            return all_gather_rows(D.to(gdev), nq_total, world), all_gather_rows(I.to(gdev), nq_total, world)
        gd = [torch.empty_like(D, device=gdev) for _ in range(world)]
        gi = [torch.empty_like(I, device=gdev) for _ in range(world)]
        dist.all_gather(gd, D.to(gdev))
        dist.all_gather(gi, I.to(gdev))
        return gd, gi

    def step():
        if graph is not None:
            graph.replay()
        else:
            local_step()
        if world > 1:  # the per-rank top-k of the batch, to every rank (RCCL all-gather)
            return gather()
        return None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    index.check()
    if graph is None:
        index.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    verified = None
    if world > 1:
        t = torch.tensor([elapsed], device=gdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the gathered result: this rank's rows as every rank received them
        gd, gi = step()
        torch.cuda.synchronize()
        rank = dist.get_rank()
        if scaling == "strong":
            s, e = shard_bounds(nq_total, rank, world)
            mine_d, mine_i = gd[s:e], gi[s:e]
        else:
            mine_d, mine_i = gd[rank], gi[rank]
        ok = torch.equal(mine_i.cpu(), I.cpu()) and torch.equal(mine_d.cpu().view(torch.int32),
                                                                 D.cpu().view(torch.int32))
        f = torch.tensor([1 if ok else 0], device=gdev, dtype=torch.int32)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        verified = bool(f.item())
    return elapsed, D, I, ncand, probe, local_step, graph, verified


def run_workload(args, data, rank, world, gpu, dev, dist, primary):
    """Build one config on one distribution, time the step, measure everything."""
    from lira_amd import PartitionedIndex, RankWorkspace, centroid_gemm, rank_nearest
    from lira_amd.distributed import shard_bounds
    from lira_amd.synthetic import CONFIGS, LATENT_DIM, N_MUL, workload

    N, d, B, nprobe, k, metric, nq_default = CONFIGS[args.config]
    n_mul = N_MUL.get(args.config, 1)
    nq_job = args.nq or nq_default
    opts = parse_opts(args.opt, args.config)
    t0 = time.time()
    x, centres, assign, make_queries = workload(args.config, args.seed, dev, data)
    index = PartitionedIndex(d, metric, gpu, **opts).build(assign if assign.dim() == 2 else assign[:, None],
                                                           x, B)  # device CSR (search.cpp:366-404)
    del assign
    if args.scaling == "strong":
        q_all = make_queries(nq_job, args.seed + 101)
        s, e = shard_bounds(nq_job, rank, world)
        q = q_all[s:e].contiguous()
        del q_all
    else:
        q = make_queries(nq_job, args.seed + 101 + 7919 * rank)
    nq = q.shape[0]
    torch.cuda.synchronize()
    sizes = np.asarray(index.list_sizes)
    log(f"[rank {rank}] built {args.config}/{data}: N={N} n_mul={n_mul} d={d} B={B} lists "
        f"{int(sizes.min())}..{int(sizes.max())} in {time.time() - t0:.1f}s, index "
        f"{index.memory_bytes() / 1e9:.1f} GB, {nq} queries/rank")

    gdev = dev if args.backend == "nccl" else torch.device("cpu")
    kernel = index.describe(nq, nprobe, k)
    elapsed, D, I, ncand, probe, local_step, graph, verified = time_batch(
        args, index, q, centres, nprobe, k, world, dist, gdev, nq_job, args.scaling)
    if graph is not None:  # per-phase kernel times: the same step launched one by one, untimed
        index.set_profiling(True)
        for _ in range(args.steps):
            local_step()
        torch.cuda.synchronize()
    prof = index.profile_read()
    index.set_profiling(False)
    other = None
    if world > 1:  # the other scaling mode on the same index: a fixed batch split over ranks, or a batch each
        om = "strong" if args.scaling == "weak" else "weak"
        if om == "strong":
            q_all = make_queries(nq_job, args.seed + 101)
            s0, e0 = shard_bounds(nq_job, rank, world)
            qo = q_all[s0:e0].contiguous()
            del q_all
        else:
            qo = make_queries(nq_job, args.seed + 101 + 7919 * rank)
        el_o, *_, ver_o = time_batch(args, index, qo, centres, nprobe, k, world, dist, gdev, nq_job, om)
        index.set_profiling(False)
        n_o = nq_job if om == "strong" else nq_job * world
        other = {"scaling": om, "value": n_o * args.steps / el_o, "unit": "queries/s",
                 "ms_per_step": el_o / args.steps * 1e3, "queries_per_step": n_o,
                 "queries_per_rank": int(qo.shape[0]), "allgather_verified": ver_o}
        del qo
    calls = max(1, prof["calls"])
    scan_ms, merge_ms, plan_ms = prof["scan_ms"] / calls, prof["merge_ms"] / calls, prof["plan_ms"] / calls
    nq_all = nq_job if args.scaling == "strong" else nq_job * world
    out = {"data": data, "value": nq_all * args.steps / elapsed, "unit": "queries/s", "other_scaling": other,
           "allgather_verified": verified,
           "ms_per_step": elapsed / args.steps * 1e3, "queries_per_rank": nq, "kernel": kernel,
           "launch": "hip_graph" if graph is not None else "stream",
           "index_bytes": index.memory_bytes(), "n_mul": n_mul, "index_options": opts,
           "kernels_ms_per_step": {"plan": plan_ms, "scan": scan_ms, "merge": merge_ms}}
    if rank != 0:
        return out

    # ---- scan work counters (one untimed step) ---------------------------------
    index.set_stats(True)
    local_step()  # (rank 0 only from here on: no collectives)
    work = index.stats_read()
    index.set_stats(False)

    def event_ms(fn, reps=20):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    if args.sweep and world == 1:
        out["sweep"] = sweep_options(args, index, local_step, D, I, nq, nprobe, k)

    ws = RankWorkspace(max(1, nq), B, dev)
    out["kernels_ms_per_step"]["rank_nearest"] = event_ms(
        lambda: rank_nearest(q, centres, nprobe, out=probe, workspace=ws))

    # ---- roofline of the scan kernel (one launch = one step's batch) ------------
    cand = int(ncand.sum().item())
    dpad = (d + 31) // 32 * 32
    qr = int(kernel.split("QR=")[1].split()[0]) if "QR=" in kernel else 64
    hh = "hi-q" in kernel  # hi x hi: 1 product per dim (qh x xh), hi parts of x and q staged
    split = "split-bf16" in kernel or hh
    hix = "hi-x" in kernel  # hi-only x: 2 products per dim (qh, ql) x xh, half the X bytes
    kname = kernel.split()[0]
    if kname in ("k_screen_m", "k_screen_r"):
        # (row, cand) pairs x dpad x products x 2
        flops = work["chunks_computed"] * dpad * (2 if hh else 4 if hix else 8 if split else 2)
        mfma_peak = MFMA_BF16_PEAK_TFLOPS if split else MFMA_F32_PEAK_TFLOPS
        mfma_what = "bf16 MFMA" if split else "fp32 MFMA"
    else:
        flops = work["chunks_computed"] * dpad * 2
        mfma_peak, mfma_what = MFMA_F32_PEAK_TFLOPS, "fp32 VALU (v_pk_fma_f32)"
    if kname == "k_screen_r":
        # L2 -> VGPR bytes per launch: per computed tile (64 candidates) their hi parts + xadj
        # (the work counter "blocks" counts tiles for this kernel)
        staged = work["blocks"] * (64 * dpad * 2 + 256)
        st_name, st_peak = "l2_vgpr", L2_PEAK_GBS
        st_what = "bytes loaded L2/MALL -> VGPRs (x hi parts + xadj per computed tile; queries from LDS)"
    else:
        # L2 -> LDS bytes (LDS-DMA) per launch: X (256 candidates), Q (qr rows), xadj
        staged = work["blocks"] * (256 * dpad * (2 if hix else 4) + qr * dpad * (2 if hh else 4) + 1024)
        st_name, st_peak = "l2_lds", L2LDS_PEAK_GBS
        st_what = "bytes staged L2/MALL -> LDS by LDS-DMA (tiles + query chunk + xadj per computed block)"
    traffic, pmc_src = None, None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_scan_{args.config}_{data}.json")
    if os.path.exists(pmc_path):
        try:
            rec = json.load(open(pmc_path))
            if rec.get("kernel_desc") == kernel and rec.get("nq") == nq:
                traffic, pmc_src = rec.get("hbm_bytes_per_launch"), os.path.relpath(pmc_path, ROOT)
        except Exception:
            traffic = None
    sec = scan_ms * 1e-3
    cands = {
        "mfma": {"achieved": flops / sec / 1e12, "peak": mfma_peak, "unit": "TFLOP/s",
                 "what": f"executed {mfma_what} flops of the screen (work counters x dpad x products)",
                 "flops_per_launch": flops},
        st_name: {"achieved": staged / sec / 1e9, "peak": st_peak, "unit": "GB/s", "what": st_what,
                  "bytes_per_launch": staged},
    }
    if traffic:
        cands["hbm"] = {"achieved": traffic / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "what": "HBM bytes from rocprofv3 PMC (2 FETCH_SIZE + WRITE_SIZE, gfx950 correction)",
                        "source": pmc_src}
    for c in cands.values():
        c["frac"] = c["achieved"] / c["peak"]
    binding = max(cands, key=lambda n: cands[n]["frac"])
    bc = cands[binding]
    eff_bytes = cand * d * 4 + nq * (4 * d + 12 * k)  # SURVEY 8(d) per-launch algorithmic bytes
    out["roofline"] = {
        "bound": "mfma" if binding == "mfma" else "hbm", "binding": binding,
        "achieved": bc["achieved"], "peak": bc["peak"], "unit": bc["unit"], "frac": bc["frac"],
        "traffic": traffic, "kernel": kernel, "kernel_ms": scan_ms, "candidates": cands,
        "effective_survey_8d": {
            "bytes_per_launch": eff_bytes, "GBps": eff_bytes / sec / 1e9,
            "note": "SURVEY 8(d) bytes (every probed candidate once per query) / scan time: NOT a "
                    "roofline -- the partition-major scan reads a candidate once per query block and "
                    "skips or screens most of them; reported for continuity only"},
        "work": {"blocks_computed": work["blocks"], "blocks_skipped": work["blocks_skipped"],
                 # (the plan filter's counters exist only when the screened path ran alone)
                 "pairs_pruned_plan": work.get("pairs_pruned_plan"),
                 "candidates_pruned_plan": work.get("candidates_pruned_plan"),
                 "blocks_pruned_plan": (work["candidates_pruned_plan"] / (qr * 256.0)
                                        if "candidates_pruned_plan" in work else None),
                 "blocks_unit": f"tiles of 64 candidates x {qr} rows" if kname == "k_screen_r"
                 else "blocks of 256 candidates x qr rows",
                 "blocks_pruned_plan_note": "(query, candidate) pairs the plan's partition filter removed, in "
                                            "units of one screen block (qr query rows x 256 candidates); "
                                            "blocks_skipped = blocks the in-kernel triangle test skipped",
                 "pairs_screened": work["chunks_computed"], "survivors": work["survivors"],
                 "rechecked": work["rechecked"], "rescans": work["rescans"],
                 "rechecked_per_query": work["rechecked"] / max(1, nq)},
    }
    out["candidates_per_query"] = cand / max(1, nq)

    if primary:
        gemm_ms = event_ms(lambda: centroid_gemm(q, centres))
        out["rank_gemm"] = {"kernel": "k_centroid_gemm (v_mfma_f32_32x32x2_f32)", "ms": gemm_ms,
                            "achieved": 2.0 * nq * B * d / (gemm_ms * 1e-3) / 1e12, "peak": MFMA_F32_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "flops": 2 * nq * B * d}
        out["rank_gemm"]["frac"] = out["rank_gemm"]["achieved"] / MFMA_F32_PEAK_TFLOPS
    # the same batch through the all-exact kernel (every candidate in
    # search.cpp's arithmetic): its time, and its output must equal the
    # screened path's bit for bit on the whole batch
    if index.has_tiles and not args.no_exact:
        De, Ie, nce = torch.empty_like(D), torch.empty_like(I), torch.empty_like(ncand)
        index.search(q, probe, k, dedup=True, out=(De, Ie, nce), exact=True)
        index.set_profiling(True)
        for _ in range(3):
            index.search(q, probe, k, dedup=True, out=(De, Ie, nce), exact=True)
        torch.cuda.synchronize()
        pe = index.profile_read()
        index.set_profiling(False)
        ex_ms = pe["scan_ms"] / max(1, pe["calls"])
        out["exact_kernel"] = {"kernel": index.describe(nq, nprobe, k, exact=True), "scan_ms": ex_ms,
                               "same_output_full_batch": bool(torch.equal(I, Ie) and torch.equal(
                                   D.view(torch.int32), De.view(torch.int32))),
                               "screen_speedup": ex_ms / scan_ms}

    # ---- parity (oracle on a sample) and recall@k (exhaustive, GPU) -------------
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    met = oracle.IP if metric == "inner_product" else oracle.L2
    big = args.config == "bigann100m"  # the index (2e8 rows) is not copied to the host
    ns = min(args.recall_sample if not big else min(args.recall_sample, 32), nq)
    rows = np.r_[0:ns // 2, nq - (ns - ns // 2):nq]
    cache = {}

    def lists(b):
        if b not in cache:
            cache[b] = index.list_ids(b)
        return cache[b]

    qh, ph = q.cpu().numpy(), probe.cpu().numpy()
    if big:
        Do, Io = oracle_sample(oracle, index, x, q, probe, rows, k, metric, lists)
        host = None
    else:
        off = np.zeros(B + 1, dtype=np.int64)
        off[1:] = np.cumsum(sizes)
        ids_h = np.concatenate([lists(b) for b in range(B)])
        host = (off, ids_h, x.cpu().numpy()[ids_h])
        oracle.set_threads(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0)))
        Do, Io, _ = oracle.scan_topk(qh[rows], *host, ph[rows], k, met, index.max_replicas)
    Ig, Dg = I.cpu().numpy()[rows], D.cpu().numpy()[rows]
    out["parity_sample"] = int(len(rows))
    out["parity_bit_exact"] = bool(np.array_equal(Io, Ig) and np.array_equal(Do.view(np.uint32),
                                                                              Dg.view(np.uint32)))
    qr_s = q[torch.from_numpy(rows).to(dev)].contiguous()
    allp = torch.arange(B, dtype=torch.int32, device=dev).repeat(len(rows), 1)
    _, Igt, _ = index.search(qr_s, allp, k, dedup=True)  # ground truth: every partition probed
    Igt = Igt.cpu().numpy()
    out["recall_at_k"] = float(np.mean([len(set(Ig[i]) & set(Igt[i])) / k for i in range(len(rows))]))
    out["recall_gate"] = out["recall_at_k"] >= 0.95
    out["recall_note"] = f"{len(rows)} queries vs exhaustive top-{k} (all {B} partitions probed, same kernel)"
    if data == "uniform":
        out["recall_note"] += (" -- uniform i.i.d. data has no cluster structure, so nprobe << B cannot reach the "
                               "0.95 gate (SURVEY.md 7, hard part 7): a throughput and parity workload")

    # ---- CPU baseline: the oracle (search.cpp's scan + top-k in its sequential
    # fp32 arithmetic, one query per thread, OpenMP over queries) on the same
    # batch and probe lists, timed on the host alone (inputs already in memory)
    if primary and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
        if host is not None:
            oracle.set_threads(1)
            pilot = np.arange(min(16, nq))
            tp = time.perf_counter()
            oracle.scan_topk(qh[pilot], *host, ph[pilot], k, met, index.max_replicas)
            st_qps = len(pilot) / max(time.perf_counter() - tp, 1e-9)
            n_cpu = int(min(nq, max(threads, st_qps * threads * 15.0)))  # ~15 s of work
            oracle.set_threads(threads)
            tc = time.perf_counter()
            oracle.scan_topk(qh[:n_cpu], *host, ph[:n_cpu], k, met, index.max_replicas)
            cpu_s = time.perf_counter() - tc
        else:  # per-query sub-CSRs prepared first (3 GB each), then only the scans are timed
            from concurrent.futures import ThreadPoolExecutor
            n_cpu = min(8, nq)  # (one query's lists are 3-8 GB on the host)
            prep = []
            for i in range(n_cpu):
                ls = [lists(int(b)) for b in ph[i] if b >= 0]
                o = np.zeros(len(ls) + 1, dtype=np.int64)
                o[1:] = np.cumsum([len(l) for l in ls])
                vv = np.concatenate([x[torch.from_numpy(l).to(dev).long()].cpu().numpy() for l in ls])
                prep.append((qh[i:i + 1], o, np.concatenate(ls).astype(np.int32), vv,
                             np.arange(len(ls), dtype=np.int32)[None, :]))
            oracle.set_threads(1)
            tp = time.perf_counter()
            oracle.scan_topk(*prep[0], k, met, index.max_replicas)
            st_qps = 1.0 / max(time.perf_counter() - tp, 1e-9)
            threads = min(threads, n_cpu)
            tc = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(lambda a: oracle.scan_topk(*a, k, met, index.max_replicas), prep))
            cpu_s = time.perf_counter() - tc
            prep_b = [(a[0], a[1], a[2], a[3], a[4]) for a in prep]
            del prep
        scalar = {
            "value": n_cpu / cpu_s, "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{n_cpu} queries of the same batch and probe lists, scan + top-k (oracle/lira_oracle.c "
                      f"= search.cpp:471-514's sequential fp32 arithmetic), one query per thread",
            "seconds": cpu_s, "single_thread_qps": st_qps,
            "nproc_linear_estimate_qps": st_qps * (os.cpu_count() or 1)}
        # faiss-like blocked BLAS form (the stronger CPU; it is what value reports)
        ip = metric == "inner_product"
        if host is not None:
            nb, bs, Db, Ib = time_blas(qh, ph, host, k, ip, threads)
            gI = I[:nb].cpu().numpy()
        else:
            nb, bs, acc = len(prep_b), 0.0, []
            torch.set_num_threads(threads)
            for a in prep_b:
                tc = time.perf_counter()
                acc.append(blas_scan_topk(*a, k, ip)[1])
                bs += time.perf_counter() - tc
            Ib, gI = np.concatenate(acc), I[:nb].cpu().numpy()
        agree = float(np.mean([len(set(Ib[i]) & set(gI[i])) / k for i in range(nb)]))
        blas_qps = nb / bs
        out["cpu_baseline"] = {
            "value": nb / bs, "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{nb} queries of the same batch and probe lists: faiss-like blocked sgemm + top-k "
                      f"(torch CPU, {threads} threads; approximates faiss IndexFlat.search's BLAS path, "
                      f"LIRA_smallscale.py:168) -- bench.py:blas_scan_topk",
            "seconds": bs, "topk_agreement_with_gpu": agree,
            "cores_of_nproc": f"{threads} of {os.cpu_count()}", "nproc": os.cpu_count(),
            "cpu_model": cpu_model(), "scalar_port": scalar,
            "note": "cores = threads used = the box's allotted CPU share (OMP_NUM_THREADS); nproc counts "
                    "the whole machine (not all of it is ours); scalar_port = search.cpp's own one-query-"
                    "per-thread form; nproc_linear_estimate = its single-thread QPS x nproc (not measured); "
                    "value = the faster of the two forms (BLAS loses on BIGANN's 7 M candidates per query)"}
        if scalar["value"] > blas_qps:  # report the stronger CPU form as the baseline, keep both
            cb = out["cpu_baseline"]
            cb["blas_form"] = {"value": blas_qps, "sample": cb["sample"], "seconds": bs,
                               "topk_agreement_with_gpu": agree}
            cb.update(value=scalar["value"], sample=scalar["sample"], seconds=scalar["seconds"])
    # ---- the MLP-probed search.cpp pipeline, N = 1 ---------------
    if primary and world == 1 and B <= 256 and not args.no_pipeline:
        out["pipeline"] = time_pipeline(args, oracle, index, x, centres, q, make_queries, k, nprobe, metric,
                                        host, rows, Igt, dev)
    del index, x
    return out


def run_partition_shard(args, data, rank, world, gpu, dev, dist):
    """--shard partitions: this rank's buckets only, the whole batch, all-gather +
    device k-way merge inside the timed step.  Checked after the timed loop: each
    rank's own result against the oracle on a sample (its own lists), the merge
    against lira_merge_shards' numpy restatement on that sample, and (configs whose
    full index fits beside the shard) the whole batch against a full index on rank 0."""
    from lira_amd import PartitionedIndex, RankWorkspace, rank_nearest
    from lira_amd.distributed import bucket_sizes, merge_shards, partition_owners, shard_assignment
    from lira_amd.synthetic import CONFIGS, N_MUL, workload
    N, d, B, nprobe, k, metric, nq_default = CONFIGS[args.config]
    n_mul = N_MUL.get(args.config, 1)
    nq = args.nq or nq_default
    opts = parse_opts(args.opt, args.config)
    t0 = time.time()
    x, centres, assign, make_queries = workload(args.config, args.seed, dev, data)
    a2 = assign if assign.dim() == 2 else assign[:, None]
    del assign
    sizes_all = bucket_sizes(a2, B)
    owners = partition_owners(sizes_all, world)
    mine = shard_assignment(a2, owners, rank)
    if args.config != "bigann100m":
        a_full = a2
    else:
        a_full = None
        del a2
    index = PartitionedIndex(d, metric, gpu, **opts).build(mine, x, B)
    del mine
    q = make_queries(nq, args.seed + 101)  # the same batch on every rank
    torch.cuda.synchronize()
    owned_rows = int(sizes_all[owners == rank].sum())
    log(f"[rank {rank}] partition shard {args.config}/{data}: {int((owners == rank).sum())} of {B} buckets, "
        f"{owned_rows} of {int(sizes_all.sum())} list rows, index {index.memory_bytes() / 1e9:.1f} GB, "
        f"built in {time.time() - t0:.1f}s")
    gdev = dev if args.backend == "nccl" else torch.device("cpu")
    ws = RankWorkspace(max(1, nq), B, dev)
    probe = torch.empty((nq, nprobe), dtype=torch.int32, device=dev)
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    ncand = torch.empty(nq, dtype=torch.int64, device=dev)
    Dall = torch.empty((world, nq, k), dtype=torch.float32, device=gdev)
    Iall = torch.empty((world, nq, k), dtype=torch.int64, device=gdev)
    Dm = torch.empty((nq, k), dtype=torch.float32, device=dev)
    Im = torch.empty((nq, k), dtype=torch.int64, device=dev)

    def local_step():
        rank_nearest(q, centres, nprobe, out=probe, workspace=ws)
        index.search(q, probe, k, dedup=True, out=(D, I, ncand))

    graph = None
    if args.graph:
        for _ in range(2):
            local_step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            local_step()
        torch.cuda.synchronize()

    def step():
        if graph is not None:
            graph.replay()
        else:
            local_step()
        if world == 1:
            return D, I
        if args.backend == "nccl":
            dist.all_gather_into_tensor(Dall, D)
            dist.all_gather_into_tensor(Iall, I)
            merge_shards(Dall, Iall, metric, True, out=(Dm, Im))
        else:
            gd = [torch.empty((nq, k), dtype=torch.float32) for _ in range(world)]
            gi = [torch.empty((nq, k), dtype=torch.int64) for _ in range(world)]
            dist.all_gather(gd, D.cpu())
            dist.all_gather(gi, I.cpu())
            merge_shards(torch.stack(gd).to(dev), torch.stack(gi).to(dev), metric, True, out=(Dm, Im))
        return Dm, Im

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    index.check()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], device=gdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    Dr, Ir = step()  # the merged result (world > 1: every rank's shard in it)
    Dr, Ir = Dr.clone(), Ir.clone()
    torch.cuda.synchronize()
    # per-phase kernel times of this rank (the same step launched one by one, untimed)
    index.set_profiling(True)
    for _ in range(args.steps):
        local_step()
    torch.cuda.synchronize()
    prof = index.profile_read()
    index.set_profiling(False)
    calls = max(1, prof["calls"])
    merge_ms, Dp, Ip = None, None, None
    if world > 1:  # every rank's own (nq, k) result, gathered once more for the checks
        if args.backend == "nccl":
            dist.all_gather_into_tensor(Dall, D)
            dist.all_gather_into_tensor(Iall, I)
            Dst, Ist = Dall, Iall
        else:
            gd = [torch.empty((nq, k), dtype=torch.float32) for _ in range(world)]
            gi = [torch.empty((nq, k), dtype=torch.int64) for _ in range(world)]
            dist.all_gather(gd, D.cpu())
            dist.all_gather(gi, I.cpu())
            Dst, Ist = torch.stack(gd).to(dev), torch.stack(gi).to(dev)
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            merge_shards(Dst, Ist, metric, True, out=(Dm, Im))
        e1.record(s)
        torch.cuda.synchronize()
        merge_ms = e0.elapsed_time(e1) / 20
        Dp, Ip = Dst.cpu().numpy(), Ist.cpu().numpy()

    # ---- checks (after timing): own shard vs oracle sample, merge restatement, full index
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    ns = min(32 if args.config == "bigann100m" else args.recall_sample, nq)
    rows = np.r_[0:ns // 2, nq - (ns - ns // 2):nq]
    cache = {}

    def lists(b):
        if b not in cache:
            cache[b] = index.list_ids(b)
        return cache[b]

    Do, Io = oracle_sample(oracle, index, x, q, probe, rows, k, metric, lists)
    own_ok = bool(np.array_equal(Io, I.cpu().numpy()[rows]) and
                  np.array_equal(Do.view(np.uint32), D.cpu().numpy()[rows].view(np.uint32)))
    merge_ok, full_ok = None, None
    if world > 1:
        Dref, Iref = oracle.merge_shards(Dp[:, rows], Ip[:, rows], metric == "inner_product", True, k)
        merge_ok = bool(np.array_equal(Iref, Ir.cpu().numpy()[rows]) and
                        np.array_equal(Dref.view(np.uint32), Dr.cpu().numpy()[rows].view(np.uint32)))
        flags = torch.tensor([int(own_ok), int(merge_ok)], dtype=torch.int32, device=gdev)
        dist.all_reduce(flags, op=dist.ReduceOp.MIN)
        own_ok, merge_ok = bool(flags[0].item()), bool(flags[1].item())
    if rank == 0 and a_full is not None:
        full = PartitionedIndex(d, metric, gpu, **opts).build(a_full, x, B)
        Df, If, _ = full.search(q, probe, k, dedup=True)
        full_ok = bool(torch.equal(If, Ir) and torch.equal(Df.view(torch.int32), Dr.view(torch.int32)))
        del full
    out = {"data": data, "value": nq * args.steps / elapsed, "unit": "queries/s", "ms_per_step": elapsed / args.steps * 1e3,
           "queries_per_rank": nq, "kernel": index.describe(nq, nprobe, k),
           "launch": "hip_graph" if graph is not None else "stream",
           "index_bytes": index.memory_bytes(), "n_mul": n_mul, "index_options": opts,
           "kernels_ms_per_step": {"plan": prof["plan_ms"] / calls, "scan": prof["scan_ms"] / calls,
                                   "merge": prof["merge_ms"] / calls, "merge_shards": merge_ms},
           "partition_shard": {"buckets_owned": int((owners == rank).sum()), "rows_owned": owned_rows,
                               "rows_total": int(sizes_all.sum()),
                               "rows_per_rank": [int(sizes_all[owners == r].sum()) for r in range(world)],
                               "own_shard_vs_oracle_sample": own_ok, "merge_vs_restatement_sample": merge_ok,
                               "merged_equals_full_index": full_ok, "sample_rows": int(len(rows)),
                               "note": "rank 0's figures; every rank ranks and scans the whole batch against its "
                                       "own buckets, then all-gather (RCCL) + lira_merge_shards inside the timed "
                                       "step; merged_equals_full_index: whole batch vs a full index on rank 0 "
                                       "(None for BIGANN: the full index does not fit beside the shard)"}}
    del index, x
    return out


def sweep_options(args, index, local_step, D, I, nq, nprobe, k):
    """Per option value: scan/merge/plan ms (HIP events, `args.steps` steps) and
    whether the batch's output is bit-identical to the default run's."""
    D0, I0 = D.clone(), I.clone()
    rows = []
    variants = []  # "a=1,2" -> two variants; "a=1 b=2" -> one variant setting both
    for spec in args.sweep:
        sets = [t.partition("=") for t in spec.split()]
        if len(sets) == 1:
            variants += [[(sets[0][0], int(v))] for v in sets[0][2].split(",")]
        else:
            variants.append([(n, int(v)) for n, _, v in sets])
    for var in variants:
        old = [(n, index.get_option(n)) for n, _ in var]
        for n, v in var:
            index.set_option(n, v)
        tag = " ".join(f"{n}={v}" for n, v in var)
        try:
            local_step()
            torch.cuda.synchronize()
            index.set_profiling(True)
            for _ in range(args.steps):
                local_step()
            torch.cuda.synchronize()
            pr = index.profile_read()
            index.set_profiling(False)
            c = max(1, pr["calls"])
            row = {"options": tag, "kernel": index.describe(nq, nprobe, k),
                   "scan_ms": pr["scan_ms"] / c, "merge_ms": pr["merge_ms"] / c, "plan_ms": pr["plan_ms"] / c,
                   "same_output": bool(torch.equal(I, I0) and torch.equal(D.view(torch.int32), D0.view(torch.int32)))}
        except RuntimeError as e:
            index.set_profiling(False)
            row = {"options": tag, "error": str(e)[:200]}
        log(f"sweep {tag}: {row}")
        rows.append(row)
        for n, v in old:
            index.set_option(n, v)
    local_step()
    return rows


def time_pipeline(args, oracle, index, x, centres, q, make_queries, k, nprobe, metric, host, rows, Igt, dev):
    """search.cpp:424-514 per batch: exact distances + standardise (one HIP
    kernel) -> MLP_2_Input (PyTorch-ROCm) -> score >= 0.5 with argmax fallback
    (lira_select_probes), nearest probed centroid first (lira_order_probes) ->
    scan + top-k, eagerly and as one replayed HIP graph.
    The MLP is fitted (untimed) to score each query's nprobe nearest centroids,
    standing in for LIRA's kNN-label training (out of scope)."""
    from lira_amd import centroid_dist
    from lira_amd.probing import MLP_2_Input, fit_probe_to_nearest, standard_scaler
    from lira_amd.search import ProbePipeline
    nq, d = q.shape
    B = centres.shape[0]
    met = oracle.IP if metric == "inner_product" else oracle.L2
    mean, scale = standard_scaler(centroid_dist(x[:65536].contiguous(), centres))  # data-side (utils.py:120-180)
    model = MLP_2_Input(B, d, B).to(dev)

    def batch(n, it):
        qb = make_queries(n, args.seed + 5000 + it)
        return centroid_dist(qb, centres, mean, scale), qb

    tf = time.perf_counter()
    fit_probe_to_nearest(model, batch, nprobe, steps=300, batch=4096)
    fit_s = time.perf_counter() - tf
    pipe = ProbePipeline(index, centres, mean, scale, model, nq, k, 0.5, dedup=True, expect_probes=nprobe)
    pipe.q.copy_(q)
    pipe.run()
    torch.cuda.synchronize()

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    for _ in range(args.warmup):
        pipe.run()
    eager_s = timed(pipe.run, args.steps)
    I_e, D_e = pipe.I.clone(), pipe.D.clone()
    pipe.capture()
    for _ in range(args.warmup):
        pipe.replay()
    graph_s = timed(pipe.replay, args.steps)
    same = bool(torch.equal(pipe.I, I_e) and torch.equal(pipe.D.view(torch.int32), D_e.view(torch.int32)))
    # per-stage device time of one eager pass (events on the current stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    parts = {"distances": 0.0, "mlp": 0.0, "select": 0.0, "scan": 0.0}
    for _ in range(5):
        ev[0].record()
        centroid_dist(pipe.q, pipe.C, pipe.mean, pipe.scale, out=pipe.dist)
        ev[1].record()
        with torch.no_grad():
            pipe.scores.copy_(pipe.model(pipe.dist, pipe.q))
        ev[2].record()
        from lira_amd import _lib
        _lib.call("lira_select_probes", _lib.ptr(pipe.scores), nq, B, pipe.mode, 0.5,
                  pipe.max_probe, _lib.ptr(pipe.probe), _lib.ptr(pipe.nprobe), _lib.stream_ptr())
        torch.addcmul(pipe.mean, pipe.dist, pipe.scale, out=pipe.raw)  # (as ProbePipeline: nearest first)
        _lib.call("lira_order_probes", _lib.ptr(pipe.probe), nq, pipe.max_probe, _lib.ptr(pipe.raw), B,
                  _lib.stream_ptr())
        ev[3].record()
        old_hint = index.get_option("probes_hint")
        index.set_option("probes_hint", pipe.expect_probes)  # (the pipeline's own scan setting)
        index.search(pipe.q, pipe.probe, k, dedup=True, out=(pipe.D, pipe.I, pipe.ncand))
        index.set_option("probes_hint", old_hint)
        ev[4].record()
        torch.cuda.synchronize()
        for i, name in enumerate(parts):
            parts[name] += ev[i].elapsed_time(ev[i + 1]) / 5
    # parity on the sample: distances, probe selection on the pipeline's scores, scan
    qs = q.cpu().numpy()[rows]
    dist_o = oracle.centroid_dist(qs, centres.cpu().numpy(), mean.cpu().numpy(), scale.cpu().numpy())
    dist_ok = bool(np.array_equal(pipe.dist.cpu().numpy()[rows].view(np.uint32), dist_o.view(np.uint32)))
    sc = pipe.scores.cpu().numpy()[rows]
    pr, cnt = oracle.probe_threshold(sc, 0.5)
    got = pipe.probe.cpu().numpy()[rows]
    sel_ok = bool(np.array_equal(pipe.nprobe.cpu().numpy()[rows], cnt) and all(
        np.array_equal(np.sort(got[i][got[i] >= 0]), pr[i][pr[i] >= 0]) for i in range(len(rows))))
    Ig, Dg = pipe.I.cpu().numpy()[rows], pipe.D.cpu().numpy()[rows]
    if host is not None:
        Do, Io, _ = oracle.scan_topk(qs, *host, pr, k, met, index.max_replicas)
        scan_ok = bool(np.array_equal(Io, Ig) and np.array_equal(Do.view(np.uint32), Dg.view(np.uint32)))
    else:
        scan_ok = None
    recall = float(np.mean([len(set(Ig[i]) & set(Igt[i])) / k for i in range(len(rows))]))
    npb = pipe.nprobe.float().mean().item()
    return {"what": "search.cpp:424-514 on the batch: lira_centroid_dist (exact + standardise) -> MLP_2_Input "
                    "(torch) -> lira_select_probes (>= 0.5, argmax fallback) -> lira_scan_topk",
            "probe_order": "lira_order_probes: the selected set by ascending raw centroid distance",
            "value_eager": nq / eager_s, "value_graph": nq / graph_s, "unit": "queries/s",
            "ms_eager": eager_s * 1e3, "ms_graph": graph_s * 1e3, "graph_same_output": same,
            "stage_ms": parts, "max_probe": pipe.max_probe,
            "avg_nprobe": npb, "recall_at_k": recall, "parity_sample": int(len(rows)),
            "parity": {"distances_bit_exact": dist_ok, "probe_selection_exact": sel_ok, "scan_bit_exact": scan_ok},
            "mlp": f"MLP_2_Input({B}, {d}, {B}) fitted in {fit_s:.1f} s (300 Adam steps) to the nearest-{nprobe} "
                   f"indicator: synthetic stand-in for LIRA's kNN labels"}


def launch_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start the N ranks as ONE child process
    tree (torch.distributed.run, rendezvous on 127.0.0.1) and return its exit
    status.  Nothing here touches the GPU (no torch.cuda call), so the
    children own the devices."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL, tensor sharing)
    log(f"[bench] --gpus {args.gpus}: starting {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)  # gloo rehearsal: several ranks may share one GPU
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    ranks_seen = {"world_size": 1, "devices": [torch.cuda.get_device_name(dev)]}
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        got = dist.get_world_size()
        if got != args.gpus:
            log(f"error: --gpus {args.gpus} but the process group has {got} ranks")
            dist.destroy_process_group()
            sys.exit(3)
        me = {"rank": dist.get_rank(), "local_rank": local, "device": gpu,
              "name": torch.cuda.get_device_name(dev), "pci_bus": torch.cuda.get_device_properties(dev).pci_bus_id,
              "host": platform.node()}
        seen = [None] * got
        dist.all_gather_object(seen, me)
        ranks_seen = {"world_size": got, "backend": args.backend, "ranks": seen,
                      "distinct_gpus": len({(r["host"], r["pci_bus"]) for r in seen})}
    elif args.gpus != 1:
        log(f"error: --gpus {args.gpus} under WORLD_SIZE={world}")
        sys.exit(3)
    from lira_amd.synthetic import CONFIGS, LATENT_DIM

    N, d, B, nprobe, k, metric, nq_default = CONFIGS[args.config]
    if args.shard == "partitions":
        args.scaling = "strong"  # one batch over the ranks' buckets
        head = run_partition_shard(args, args.data, rank, world, gpu, dev, dist)
    else:
        head = run_workload(args, args.data, rank, world, gpu, dev, dist, primary=True)
    contrast = contrast_u = None
    if args.contrast == "auto" and world == 1 and args.config in ("sift1m", "gist1m") and args.shard == "queries":
        torch.cuda.empty_cache()
        other = "latent" if args.data != "latent" else "mixture"
        contrast = run_workload(args, other, rank, world, gpu, dev, dist, primary=False)
        if args.config == "sift1m" and args.data != "uniform":  # north_star's literal random-float vectors
            torch.cuda.empty_cache()
            contrast_u = run_workload(args, "uniform", rank, world, gpu, dev, dist, primary=False)

    if rank == 0:
        nq_job = args.nq or nq_default
        line = {
            "metric": "queries/sec at recall@10>=0.95 (SIFT1M d=128, B=64, nprobe=8), 1/2/4/8 GPU"
            if args.config == "sift1m" else f"queries/sec ({args.config})",
            "value": head["value"],
            "unit": "queries/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "accumulation": "fma (LIRA_SCAN_FMA, tolerance variant)" if args.fma
            else "split-bf16 MFMA screen (hi/lo bf16 parts, fp32 accumulation) under a rigorous error "
                 "bound + exact re-check in search.cpp's sequential fp32 sub/mul/add: bit-exact",
            "data": (f"synthetic latent (intrinsic dim {LATENT_DIM[args.config]}, k-means partitions)"
                     if args.data == "latent" else
                     "synthetic uniform random floats U[0,1)^d (k-means partitions)" if args.data == "uniform" else
                     "synthetic Gaussian mixture (sigma 0.35, separated clusters, nearest-centre partitions)"),
            "config": {"workload": args.config, "N": N, "d": d, "B": B, "nprobe": nprobe, "k": k,
                       "metric": metric, "n_mul": head["n_mul"],
                       "queries_per_step": nq_job * (world if args.scaling == "weak" else 1),
                       "queries_per_rank": head["queries_per_rank"],
                       "parallelism": f"query-shard x{world} (index replicated)" if args.shard == "queries"
                       else f"partition-shard x{world} (each rank its buckets' lists; all-gather + k-way merge)"},
            "other_scaling": head.get("other_scaling"),
            "allgather_verified": head.get("allgather_verified"),
            "roofline": head.get("roofline"),
            "cpu_baseline": head.get("cpu_baseline"),
            **{key: head[key] for key in ("kernels_ms_per_step", "kernel", "index_bytes", "index_options", "pipeline",
                                          "rank_gemm", "exact_kernel", "candidates_per_query", "parity_sample",
                                          "parity_bit_exact", "recall_at_k", "recall_gate", "recall_note",
                                          "partition_shard", "sweep")
               if key in head},
            "contrast_data": contrast,
            "contrast_uniform": contrast_u,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()  # (rank 0's untimed legs above run without collectives)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
