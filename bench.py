"""Benchmark of LIRA's query-time hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config sift1m]

One step = one pass of the hot path over one batch of synthetic queries on
every rank: MFMA ranking GEMM + exact nprobe boundary re-check
(lira_rank_nearest) -> batched scan + exact top-k (lira_scan_topk) -> for
N > 1 an RCCL all-gather of the per-rank top-k (the query batch is sharded,
every rank holds a full index replica).  Inputs are resident in
HBM before the timed region.  Rank 0 prints ONE JSON line (the bench contract).

Multi-GPU: launched as `python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N ...`; per-rank work is fixed (weak scaling), value = queries
of all ranks / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lira-ann-search_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_F32_PEAK_TOPS = 78.64   # non-FMA fp32 lane ops/s: 157.3 TFLOP/s counts an FMA as 2
MFMA_F32_PEAK_TFLOPS = 157.3  # v_mfma_f32_32x32x2_f32 dense peak (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA peak, 16 x the f32 rate (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="sift1m", choices=["sift1m", "gist1m", "deep10m", "bigann100m"])
    ap.add_argument("--nq", type=int, default=None, help="queries per rank per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1024)
    ap.add_argument("--recall-sample", type=int, default=100)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--fma", action="store_true",
                    help="LIRA_SCAN_FMA accumulation (tolerance variant, not the reference's rounding)")
    ap.add_argument("--data", default="mixture", choices=["latent", "mixture"],
                    help="synthetic distribution (lira_amd/synthetic.py): mixture = SURVEY 8(d)'s "
                         "Gaussian mixture (default; separated clusters, so exact pruning skips most "
                         "non-nearest partitions); latent = low intrinsic dimension + k-means "
                         "partitions, recall near the metric's 0.95 point like real SIFT1M")
    ap.add_argument("--contrast", default="auto", choices=["auto", "none"],
                    help="auto: at N=1 on sift1m/gist1m also time the other distribution "
                         "(reported as contrast_data, untimed by the headline)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N>1 on one GPU")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    from lira_amd import PartitionedIndex, RankWorkspace, centroid_gemm, rank_nearest
    from lira_amd.synthetic import CONFIGS, LATENT_DIM, workload

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world != 1:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)  # gloo rehearsal: several ranks may share one GPU
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    N, d, B, nprobe, k, metric, nq_default = CONFIGS[args.config]
    nq = args.nq or nq_default
    t0 = time.time()
    # ---- synthetic index (identical on every rank: same seed) ----------------
    x, centres, assign, make_queries = workload(args.config, args.seed, dev, args.data)
    index = PartitionedIndex(d, metric, gpu).build(assign[:, None], x, B)  # device CSR (search.cpp:366-404)
    offsets = np.zeros(B + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(index.list_sizes)
    rep = index.max_replicas
    # rank-specific queries (weak scaling: each rank owns a disjoint batch)
    q = make_queries(nq, args.seed + 101 + 7919 * rank)
    torch.cuda.synchronize()
    log(f"[rank {rank}] built {args.config}: N={N} d={d} B={B} lists "
        f"{int(np.min(np.diff(offsets)))}..{int(np.max(np.diff(offsets)))} in {time.time() - t0:.1f}s")

    ws = RankWorkspace(nq, B, dev)
    probe = torch.empty((nq, nprobe), dtype=torch.int32, device=dev)
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    ncand = torch.empty(nq, dtype=torch.int64, device=dev)
    gdev = dev if args.backend == "nccl" else torch.device("cpu")
    gD = [torch.empty(D.shape, dtype=D.dtype, device=gdev) for _ in range(world)] if world > 1 else None
    gI = [torch.empty(I.shape, dtype=I.dtype, device=gdev) for _ in range(world)] if world > 1 else None

    def step():
        rank_nearest(q, centres, nprobe, out=probe, workspace=ws)
        index.search(q, probe, k, dedup=True, out=(D, I, ncand), fma=args.fma)
        if world > 1:  # the per-rank top-k of the sharded batch, to every rank
            dist.all_gather(gD, D.to(gdev))
            dist.all_gather(gI, I.to(gdev))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    index.check()
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
    prof = index.profile_read()
    index.set_profiling(False)
    if world > 1:
        t = torch.tensor([elapsed], device=gdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- scan work counters (one untimed step): what the L2 early abandon skips ---
    index.set_stats(True)
    step()
    work = index.stats_read()
    if os.environ.get("LIRA_SCAN_DEBUG"):
        print("work_raw", work, file=sys.stderr)
    index.set_stats(False)

    # ---- the ranking GEMM alone (MFMA utilisation), outside the timed region ---
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

    gemm_ms = event_ms(lambda: centroid_gemm(q, centres))
    # the same batch through the all-exact kernel (every candidate in
    # search.cpp's arithmetic; LIRA_SCAN_EXACT) into separate buffers: its time
    # is what the FMA screen is measured against, and its output must equal
    # the screened path's bit for bit on the whole batch
    De, Ie, nce = torch.empty_like(D), torch.empty_like(I), torch.empty_like(ncand)
    index.set_profiling(True)
    for _ in range(3):
        index.search(q, probe, k, dedup=True, out=(De, Ie, nce), exact=True)
    torch.cuda.synchronize()
    prof_ex = index.profile_read()
    index.set_profiling(False)
    scan_ex_ms = prof_ex["scan_ms"] / max(1, prof_ex["calls"])
    full_batch_equal = bool(torch.equal(I, Ie) and torch.equal(D.view(torch.int32), De.view(torch.int32)))
    rank_ms = event_ms(lambda: rank_nearest(q, centres, nprobe, out=probe, workspace=ws))
    gemm_tflops = 2.0 * nq * B * d / (gemm_ms * 1e-3) / 1e12

    # ---- per-launch algorithmic figures -----------------------
    cand = int(ncand.sum().item())  # candidates scanned in one launch (this rank)
    bytes_launch = cand * d * 4 + nq * (4 * d + 12 * k)
    flops_launch = cand * d * (3 if metric == "L2" else 2)
    scan_ms = prof["scan_ms"] / max(1, prof["calls"])
    merge_ms = prof["merge_ms"] / max(1, prof["calls"])
    plan_ms = prof["plan_ms"] / max(1, prof["calls"])
    achieved_gbs = bytes_launch / (scan_ms * 1e-3) / 1e9
    # Compute: the screen runs one fp32 FMA per (query row, candidate, dim) of
    # every wave-block it does not skip (padding rows of a block included);
    # the work counters give the (row, candidate) pairs screened per launch.  fp32 peak 157.3 TF is
    # the same on MFMA and VALU (v_pk_fma_f32) on MI355X.
    dpad = (d + 31) // 32 * 32
    screen_flops = 2.0 * work["chunks_computed"] * dpad  # stats[0]: (row, candidate) pairs screened
    screen_tflops = screen_flops / (scan_ms * 1e-3) / 1e12
    ex_tops = flops_launch / (scan_ex_ms * 1e-3) / 1e12
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_scan_{args.config}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    qps = world * nq * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # ---- parity + recall gate on a sample, CPU baseline (rank 0, N=1 only) ---
    extra = {}
    cpu = None
    if rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        ns = min(args.recall_sample, nq)
        xs = x.cpu().numpy()
        off = np.asarray(offsets, dtype=np.int64)
        ids_np = np.concatenate([index.list_ids(b) for b in range(B)])
        vecs = xs[ids_np]
        qs = q[:ns].cpu().numpy()
        pr = probe[:ns].cpu().numpy()
        met = oracle.IP if metric == "inner_product" else oracle.L2
        Do, Io, _ = oracle.scan_topk(qs, off, ids_np, vecs, pr, k, met, rep)
        Ig = I[:ns].cpu().numpy()
        Dg = D[:ns].cpu().numpy()
        parity = bool(np.array_equal(Io, Ig) and np.array_equal(Do.view(np.uint32), Dg.view(np.uint32)))
        if args.fma:  # tolerance variant: relative distance error and id agreement instead
            extra_fma = {"max_rel_err": float(np.max(np.abs(Dg - Do) / np.maximum(np.abs(Do), 1e-30))),
                         "id_agreement": float(np.mean(Ig == Io))}
        allp = np.tile(np.arange(B, dtype=np.int32), (ns, 1))
        _, Igt, _ = oracle.scan_topk(qs, off, ids_np, vecs, allp, k, met, rep)
        recall = float(oracle.recall_at_k(Ig, Igt, k).mean())
        extra = {"parity_sample": ns, "parity_bit_exact": parity, "recall_at_k": recall,
                 "recall_gate": recall >= 0.95}
        if args.fma:
            extra["fma_variant"] = extra_fma
        if world == 1 and not args.no_cpu_baseline:
            nc = min(args.cpu_sample, nq)
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
            threads = min(threads, 16)
            oracle.set_threads(threads)
            qc = q[:nc].cpu().numpy()
            pc = probe[:nc].cpu().numpy()
            tc = time.perf_counter()
            oracle.scan_topk(qc, off, ids_np, vecs, pc, k, met, rep)
            cpu_s = time.perf_counter() - tc
            n1 = min(64, nc)
            oracle.set_threads(1)
            t1 = time.perf_counter()
            oracle.scan_topk(qc[:n1], off, ids_np, vecs, pc[:n1], k, met, rep)
            cpu1 = time.perf_counter() - t1
            cpu = {"value": nc / cpu_s, "unit": "queries/s", "cores": threads, "kind": "port",
                   "sample": f"{nc} queries of the same batch/probe lists, scan+top-k only "
                             f"(oracle/lira_oracle.c, OpenMP over queries)",
                   "single_thread_qps": n1 / cpu1}

    # ---- the other synthetic distribution, same config and kernels (N=1) ----
    contrast = None
    if args.contrast == "auto" and world == 1 and args.config in ("sift1m", "gist1m"):
        other = "latent" if args.data == "mixture" else "mixture"
        del index, x
        torch.cuda.empty_cache()
        x2, c2, a2, mq2 = workload(args.config, args.seed, dev, other)
        idx2 = PartitionedIndex(d, metric, gpu).build(a2[:, None], x2, B)
        q2 = mq2(nq, args.seed + 101)

        def step2():
            rank_nearest(q2, c2, nprobe, out=probe, workspace=ws)
            idx2.search(q2, probe, k, dedup=True, out=(D, I, ncand), fma=args.fma)

        for _ in range(args.warmup):
            step2()
        torch.cuda.synchronize()
        idx2.set_profiling(True)
        t2 = time.perf_counter()
        for _ in range(args.steps):
            step2()
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t2
        pr2 = idx2.profile_read()
        idx2.set_profiling(False)
        # recall@k on a sample against exhaustive ground truth, and oracle parity
        off2 = np.zeros(B + 1, dtype=np.int64)
        off2[1:] = np.cumsum(idx2.list_sizes)
        ids2 = np.concatenate([idx2.list_ids(b) for b in range(B)])
        ns = min(args.recall_sample, nq)
        xs2 = x2.cpu().numpy()
        met = oracle.IP if metric == "inner_product" else oracle.L2
        qs2 = q2[:ns].cpu().numpy()
        Do2, Io2, _ = oracle.scan_topk(qs2, off2, ids2, xs2[ids2], probe[:ns].cpu().numpy(), k, met,
                                       idx2.max_replicas)
        allp = np.tile(np.arange(B, dtype=np.int32), (ns, 1))
        _, Igt2, _ = oracle.scan_topk(qs2, off2, ids2, xs2[ids2], allp, k, met, idx2.max_replicas)
        contrast = {"data": other, "value": nq * args.steps / el2, "unit": "queries/s",
                    "ms_per_step": el2 / args.steps * 1e3,
                    "scan_ms": pr2["scan_ms"] / max(1, pr2["calls"]),
                    "recall_at_k": float(oracle.recall_at_k(I[:ns].cpu().numpy(), Igt2, k).mean()),
                    "parity_bit_exact": bool(np.array_equal(Io2, I[:ns].cpu().numpy()) and np.array_equal(
                        Do2.view(np.uint32), D[:ns].cpu().numpy().view(np.uint32))),
                    "parity_sample": ns}
        del idx2, x2

    if rank == 0:
        line = {
            "metric": "queries/sec at recall@10>=0.95 (SIFT1M d=128, B=64, nprobe=8), 1/2/4/8 GPU"
            if args.config == "sift1m" else f"queries/sec ({args.config})",
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "accumulation": "fma (LIRA_SCAN_FMA, tolerance variant)" if args.fma
            else "split-bf16 MFMA screen (hi/lo bf16 parts, fp32 accumulation) under a rigorous error "
                 "bound + exact re-check in search.cpp's sequential fp32 sub/mul/add: bit-exact",
            "data": (f"synthetic latent (intrinsic dim {LATENT_DIM[args.config]}, k-means partitions)"
                     if args.data == "latent" else
                     "synthetic Gaussian mixture (sigma 0.35, separated clusters, nearest-centre partitions)"),
            "config": {"workload": args.config, "N": N, "d": d, "B": B, "nprobe": nprobe, "k": k,
                       "metric": metric, "queries_per_rank_per_step": nq,
                       "parallelism": f"query-shard x{world} (index replicated)"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_screen_m" if k <= 56 else "k_screen", "kernel_ms": scan_ms,
                         "algorithmic_bytes_per_launch": bytes_launch,
                         "hbm_actual": None if traffic is None else {
                             "achieved": traffic / (scan_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": traffic / (scan_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "source": "profiles/pmc_scan_%s.json (rocprofv3 PMC)" % args.config},
                         "compute": {"kernel": "k_screen_m<SPLIT> (v_mfma_f32_16x16x32_bf16, 4 bf16 products "
                                               "per dim) / k_screen (k > 56, fp32 VALU)",
                                     "achieved": screen_tflops, "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                     "frac": screen_tflops / MFMA_F32_PEAK_TFLOPS,
                                     "flops_executed": screen_flops,
                                     "bf16_mfma": {"achieved": 4 * screen_tflops, "peak": MFMA_BF16_PEAK_TFLOPS,
                                                   "frac": 4 * screen_tflops / MFMA_BF16_PEAK_TFLOPS,
                                                   "note": "the split form executes 4 bf16 products per "
                                                           "fp32-equivalent multiply-add"} if k <= 56 else None,
                                     "note": "fp32-equivalent: 2 x (row, candidate) pairs screened x dpad (stats[0]); "
                                             "the rest of the SURVEY 8(d) work is skipped exactly "
                                             "(triangle bound) or never needed (screen)"},
                         "exact_kernel": {"kernel": "k_scan (LIRA_SCAN_EXACT)", "scan_ms": scan_ex_ms,
                                          "valu_achieved": ex_tops, "valu_frac": ex_tops / VALU_F32_PEAK_TOPS,
                                          "valu_unit": "T lane-op/s (%d fp32 ops per candidate-dim)"
                                                       % (3 if metric == "L2" else 2),
                                          "speedup_of_screen": scan_ex_ms / scan_ms,
                                          "same_output_full_batch": full_batch_equal},
                         "work": {"blocks": work["blocks"], "blocks_skipped": work["blocks_skipped"],
                                  "survivors": work["survivors"],
                                  "rechecked": work["rechecked"], "rescans": work["rescans"],
                                  "rechecked_per_query": work["rechecked"] / nq,
                                  "rechecked_frac_of_candidates": work["rechecked"] / max(1, cand)},
                         "note": "SURVEY 8(d) algorithmic bytes = sum over queries of probed-bucket "
                                 "bytes; the partition-major scan reads a candidate tile once per "
                                 "64-query block, so that effective figure exceeds the HBM peak "
                                 "(frac > 1) while actual HBM traffic stays far below it; the "
                                 "binding resources are the fp32 MFMA rate (compute) and the "
                                 "L2->LDS staging; see DESIGN.md"},
            "kernels_ms_per_step": {"plan": plan_ms, "scan": scan_ms, "merge": merge_ms,
                                    "rank_nearest": rank_ms},
            "rank_gemm": {"kernel": "k_centroid_gemm (v_mfma_f32_32x32x2_f32)", "ms": gemm_ms,
                          "achieved": gemm_tflops, "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": gemm_tflops / MFMA_F32_PEAK_TFLOPS,
                          "flops": 2 * nq * B * d,
                          "note": "query x centroid GEMM of the ranking step (2*nq*B*d); "
                                  "rank_nearest adds the exact re-check + top-nprobe select"},
            "cpu_baseline": cpu,
            "contrast_data": contrast,
            "candidates_per_query": cand / nq,
            **extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
