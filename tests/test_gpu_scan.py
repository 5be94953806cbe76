"""GPU parity: the HIP scan + top-k (lira_scan_topk) against the golden fixtures
and the CPU oracle, bit-exact on distances and ids (search.cpp:253-269 order)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden

pytestmark = pytest.mark.gpu

GOLDEN = ["toy_l2", "toy_ip", "sift_like_redundant", "deep_like_k100_ip", "odd_dim"]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def make_index(x, d2b, n_bkt, metric, **options):
    from lira_amd import PartitionedIndex
    return PartitionedIndex.from_assignment(torch.from_numpy(x).cuda(), torch.from_numpy(d2b).cuda(),
                                            n_bkt, metric, **options)


def run(idx, q, probe, k, **kw):
    D, I, nc = idx.search(torch.from_numpy(q).cuda(), torch.from_numpy(probe).cuda(), k, **kw)
    torch.cuda.synchronize()
    idx.check()
    return D.cpu().numpy(), I.cpu().numpy(), nc.cpu().numpy()


@pytest.mark.parametrize("name", GOLDEN)
def test_golden(name):
    g = load_golden(name)
    metric = str(g["metric"])
    k = int(g["k"])
    idx = make_index(g["x"], g["data_2_bkt"], g["centroids"].shape[0], metric)
    assert idx.max_replicas == max(1, int(g["dedup_rep"]))
    D, I, nc = run(idx, g["q"], g["probe"], k, dedup=True)
    assert np.array_equal(I, g["I"])
    assert np.array_equal(bits(D), bits(g["D"]))
    assert np.array_equal(nc, g["ncand"])
    D, I, _ = run(idx, g["q"], g["probe"], k, dedup=False)
    assert np.array_equal(I, g["I_nodedup"]) and np.array_equal(bits(D), bits(g["D_nodedup"]))
    D, I, _ = run(idx, g["q"], g["probe"], k, per_partition=True, dedup=False)
    assert np.array_equal(I, g["I_part"]) and np.array_equal(bits(D), bits(g["D_part"]))


def random_case(seed, n, d, b, nq, nprobe, metric, red=0.0, uniform=False):
    rng = np.random.default_rng(seed)
    if uniform:
        x = rng.random((n, d), dtype=np.float32)
        q = rng.random((nq, d), dtype=np.float32)
        c = rng.random((b, d), dtype=np.float32)
    else:
        c = rng.standard_normal((b, d), dtype=np.float32)
        x = (c[rng.integers(0, b, n)] + 0.35 * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
        q = (c[rng.integers(0, b, nq)] + 0.35 * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
    d2b = np.full((n, 2), -1, np.int32)
    d2b[:, 0] = rng.integers(0, b, n)
    if red:
        r = rng.random(n) < red
        d2b[r, 1] = rng.integers(0, b, r.sum())
    probe = np.stack([rng.permutation(b)[:nprobe] for _ in range(nq)]).astype(np.int32)
    return x, q, d2b, probe


def check_vs_oracle(x, q, d2b, probe, b, k, metric, dedup=True):
    # every scan path: the default split-bf16 MFMA screen + exact re-check,
    # the fp32 MFMA screen (split=False), and the all-exact kernel (exact=True)
    idx = make_index(x, d2b, b, metric)
    off, ids = oracle.build_csr(d2b, b)
    vecs = oracle.gather_lists(x, off, ids)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    rep = idx.max_replicas if dedup else 0
    Do, Io, nco = oracle.scan_topk(q, off, ids, vecs, probe, k, met, rep)
    for exact, split in ((False, True), (False, False), (True, True)):
        D, I, nc = run(idx, q, probe, k, dedup=dedup, exact=exact, split=split)
        assert np.array_equal(I, Io), f"ids differ (exact={exact}, split={split})"
        assert np.array_equal(bits(D), bits(Do)), f"distances differ (exact={exact}, split={split})"
        assert np.array_equal(nc, nco)
    if k <= 56:
        for xhi in (0, 1, 2):  # hi + lo / hi-only x / hi x hi screens (wider bounds, same results)
            idx.set_option("xhi", xhi)
            D, I, nc = run(idx, q, probe, k, dedup=dedup)
            assert np.array_equal(I, Io), f"ids differ (xhi={xhi})"
            assert np.array_equal(bits(D), bits(Do)), f"distances differ (xhi={xhi})"
        idx.set_option("xhi", -1)
        # the hi x hi screen as k_screen_m (LIRA_OPT_RSCREEN = 0) where k_screen_r is the default
        idx.set_option("rscreen", 0)
        D, I, nc = run(idx, q, probe, k, dedup=dedup)
        idx.set_option("rscreen", 1)
        assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do)), "differ (rscreen=0)"
    # the merge's chunk re-scans queued for k_rescan (LIRA_OPT_RESCAN = 1) and inline (0);
    # k_screen_r without its spill lists (its full lists then re-scanned)
    for name, v in (("rescan", 1), ("rescan", 0), ("spill", 0)):
        idx.set_option(name, v)
        D, I, nc = run(idx, q, probe, k, dedup=dedup)
        idx.set_option(name, -1)
        assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do)), f"differ ({name}={v})"
    if k <= 120:
        # the compact index (no fp32 tiles: row-major + split-bf16 copies only)
        idc = make_index(x, d2b, b, metric, keep_tiles=False)
        assert not idc.has_tiles and idc.memory_bytes() < idx.memory_bytes()
        D, I, nc = run(idc, q, probe, k, dedup=dedup)
        assert np.array_equal(I, Io), "ids differ (compact index)"
        assert np.array_equal(bits(D), bits(Do)), "distances differ (compact index)"
        assert np.array_equal(nc, nco)
    return idx


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
@pytest.mark.parametrize("k", [1, 10, 64, 65, 100, 256])
def test_k_sweep(metric, k):
    x, q, d2b, probe = random_case(100 + k, 6000, 32, 12, 70, 5, metric, red=0.05)
    check_vs_oracle(x, q, d2b, probe, 12, k, metric)


@pytest.mark.parametrize("d", [1, 3, 31, 33, 96, 128, 200, 960])
def test_dims(d):
    x, q, d2b, probe = random_case(200 + d, 3000, d, 6, 33, 3, "L2")
    idx = check_vs_oracle(x, q, d2b, probe, 6, 10, "L2")
    if d > 128 and (d + 31) // 32 % 2 == 0:  # k_screen_r with the rows' hi parts streamed (LIRA_OPT_RSCREEN = 2)
        off, ids = oracle.build_csr(d2b, 6)
        vecs = oracle.gather_lists(x, off, ids)
        for metric, k in (("L2", 10), ("L2", 100), ("inner_product", 100)):
            idx2 = idx if metric == "L2" else make_index(x, d2b, 6, metric)
            idx2.set_option("rscreen", 2)
            assert idx2.describe(33, 3, k).startswith("k_screen_r"), (metric, k)
            met = oracle.IP if metric == "inner_product" else oracle.L2
            Do, Io, _ = oracle.scan_topk(q, off, ids, vecs, probe, k, met, idx2.max_replicas)
            D, I, _ = run(idx2, q, probe, k)
            assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do)), (metric, k)
            idx2.set_option("rscreen", 1)


def test_uniform_random_float_inputs():
    x, q, d2b, probe = random_case(7, 8000, 64, 16, 100, 6, "L2", uniform=True)
    check_vs_oracle(x, q, d2b, probe, 16, 10, "L2")


def test_single_query_splits_chunks():
    # tiny batch -> the planner splits buckets into chunks; results unchanged
    x, q, d2b, probe = random_case(8, 40000, 16, 4, 1, 4, "L2")
    check_vs_oracle(x, q, d2b, probe, 4, 10, "L2")
    x, q, d2b, probe = random_case(9, 40000, 16, 4, 3, 2, "inner_product", red=0.2)
    check_vs_oracle(x, q, d2b, probe, 4, 100, "inner_product")


def test_ragged_empty_and_padded_probes():
    rng = np.random.default_rng(3)
    n, d, b = 2000, 24, 10
    x = rng.standard_normal((n, d), dtype=np.float32)
    d2b = np.full((n, 1), -1, np.int32)
    # bucket sizes 0, 1, 63, 64, 65, rest random; bucket 9 empty
    sizes = [0, 1, 63, 64, 65]
    pos = 0
    for bi, s in enumerate(sizes):
        d2b[pos:pos + s, 0] = bi
        pos += s
    d2b[pos:, 0] = rng.integers(5, 9, n - pos)
    q = rng.standard_normal((50, d), dtype=np.float32)
    probe = rng.integers(-1, b, (50, 7)).astype(np.int32)
    probe[0] = -1  # a query probing nothing -> all pads
    probe[1] = [0, 0, 9, 1, -1, -1, 1]  # empty buckets + duplicate slots
    check_vs_oracle(x, q, d2b, probe, b, 10, "L2", dedup=False)
    idx = check_vs_oracle(x, q, d2b, probe, b, 70, "L2", dedup=False)
    D, I, nc = run(idx, q, probe, 10)
    assert (I[0] == -1).all() and np.isinf(D[0]).all() and nc[0] == 0


def test_out_of_range_probe_is_reported():
    from lira_amd import LiraError
    x, q, d2b, probe = random_case(4, 1000, 8, 4, 5, 2, "L2")
    idx = make_index(x, d2b, 4, "L2")
    probe[2, 1] = 4
    D, I, _ = idx.search(torch.from_numpy(q).cuda(), torch.from_numpy(probe).cuda(), 5)
    torch.cuda.synchronize()
    with pytest.raises(LiraError, match="ERANGE"):
        idx.check()
    idx.check()  # cleared


def test_empty_batch_and_idempotence():
    x, q, d2b, probe = random_case(5, 5000, 16, 8, 64, 4, "L2")
    idx = make_index(x, d2b, 8, "L2")
    D0, I0, _ = run(idx, q[:0], probe[:0], 10)
    assert D0.shape == (0, 10)
    a = run(idx, q, probe, 10)
    b_ = run(idx, q, probe, 10)
    assert np.array_equal(a[1], b_[1]) and np.array_equal(bits(a[0]), bits(b_[0]))
    # batch-order independence: each query alone gives the same row
    for i in (0, 17, 63):
        Di, Ii, _ = run(idx, q[i:i + 1], probe[i:i + 1], 10)
        assert np.array_equal(Ii[0], a[1][i]) and np.array_equal(bits(Di[0]), bits(a[0][i]))


def test_device_csr_builder_matches_search_cpp():
    from lira_amd import LiraError, PartitionedIndex
    rng = np.random.default_rng(21)
    n, b = 20000, 37
    x = rng.standard_normal((n, 12), dtype=np.float32)
    d2b = rng.integers(-1, b, (n, 3)).astype(np.int32)
    d2b[::7, 1] = d2b[::7, 0]  # a bucket repeated inside a row (search.cpp:384 uniques it)
    off, ids = oracle.build_csr(d2b, b)
    # list order (LIRA_OPT_ORDER = 0): exactly search.cpp's CSR
    idx0 = PartitionedIndex(12, "L2", order=0).build(torch.from_numpy(d2b).cuda(), torch.from_numpy(x).cuda(), b)
    assert np.array_equal(idx0.list_sizes, np.diff(off))
    for bb in range(b):
        assert np.array_equal(idx0.list_ids(bb), ids[off[bb]:off[bb + 1]])
    # default (L2): the same lists, each stored by ascending distance to its pivot
    # (the mean of its rows); ties keep list order
    idx = PartitionedIndex(12, "L2").build(torch.from_numpy(d2b).cuda(), torch.from_numpy(x).cuda(), b)
    assert np.array_equal(idx.list_sizes, np.diff(off))
    for bb in range(b):
        got, ref = idx.list_ids(bb), ids[off[bb]:off[bb + 1]]
        assert np.array_equal(np.sort(got), np.sort(ref))
        if len(ref):
            piv = x[ref].astype(np.float64).mean(0)
            rad = np.sqrt(((x[got].astype(np.float64) - piv) ** 2).sum(1)).astype(np.float32)
            assert (np.diff(rad) >= -1e-5 * (1 + rad[1:])).all()
    distinct = max(len(set(r[r >= 0])) for r in d2b)
    assert idx.max_replicas == distinct
    q = rng.standard_normal((20, 12), dtype=np.float32)
    probe = rng.integers(0, b, (20, 5)).astype(np.int32)
    D, I, _ = run(idx, q, probe, 10)
    Do, Io, _ = oracle.scan_topk(q, off, ids, x[ids], probe, 10, oracle.L2, distinct)
    assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do))
    bad = d2b.copy()
    bad[5, 0] = b
    with pytest.raises(LiraError, match="out of range"):
        PartitionedIndex(12, "L2").build(torch.from_numpy(bad).cuda(), torch.from_numpy(x).cuda(), b)


@pytest.mark.parametrize("metric,k,red", [("L2", 10, 0.3), ("inner_product", 100, 0.3), ("L2", 64, 0.0)])
def test_two_phase_pruned_scan(metric, k, red):
    # >= 32 queries per partition: the scan runs the first probe slot as its own
    # phase and prunes the rest against the published per-query bounds
    x, q, d2b, probe = random_case(300 + k, 20000, 40, 6, 600, 4, metric, red=red)
    check_vs_oracle(x, q, d2b, probe, 6, k, metric, dedup=True)
    check_vs_oracle(x, q, d2b, probe, 6, k, metric, dedup=False)
    idx = make_index(x, d2b, 6, metric)
    off, ids = oracle.build_csr(d2b, 6)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Dp, Ip = oracle.scan_per_partition(q, off, ids, oracle.gather_lists(x, off, ids), probe, k, met)
    D, I, _ = run(idx, q, probe, k, per_partition=True, dedup=False)
    assert np.array_equal(I, Ip) and np.array_equal(bits(D), bits(Dp))


@pytest.mark.parametrize("metric,k", [("L2", 10), ("inner_product", 10), ("L2", 100), ("inner_product", 100)])
def test_fma_variant_within_tolerance(metric, k):
    # LIRA_SCAN_FMA (SURVEY 7 tolerance fallback): distances within 1e-4
    # relative of search.cpp's; every returned id is a valid top-k member up to
    # that tolerance (tie-aware), and ids agree wherever the oracle's distances
    # are not near-tied.
    x, q, d2b, probe = random_case(400 + k, 20000, 96, 8, 300, 4, metric, red=0.1)
    idx = make_index(x, d2b, 8, metric)
    off, ids = oracle.build_csr(d2b, 8)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Do, Io, nco = oracle.scan_topk(q, off, ids, oracle.gather_lists(x, off, ids), probe, k, met, idx.max_replicas)
    Dk1 = oracle.scan_topk(q, off, ids, oracle.gather_lists(x, off, ids), probe, k + 1, met, idx.max_replicas)[0]
    D, I, nc = run(idx, q, probe, k, fma=True)
    assert np.array_equal(nc, nco)
    tol = 1e-4
    assert np.all(np.abs(D - Do) <= tol * np.maximum(np.abs(Do), 1e-6))
    sign = -1.0 if metric == "inner_product" else 1.0
    for r in range(q.shape[0]):
        kth = sign * Do[r, -1]
        assert len(set(I[r])) == k
        # exact distance of each returned id (oracle arithmetic) within tolerance of the k-th
        ex = oracle.scan_topk(q[r:r + 1], np.array([0, len(I[r])], np.int64), I[r].astype(np.int32),
                              x[I[r]], np.zeros((1, 1), np.int32), k, met, 0)[0][0]
        assert np.all(sign * ex <= kth + tol * abs(kth) + 1e-6)
        gap = np.abs(np.diff(Dk1[r])) > tol * np.maximum(np.abs(Dk1[r, 1:]), 1e-6)
        if gap.all():  # no near-tie inside the top k nor at its boundary
            assert np.array_equal(I[r], Io[r])


def clustered_case(seed, n, d, b, nq, nprobe, spread=3.0, sigma=0.35, ints=False):
    # well-separated clusters: pairs outside a query's own cluster pass its k-th
    # score within a few dims, so the L2 early abandon drops whole blocks
    rng = np.random.default_rng(seed)
    c = spread * rng.standard_normal((b, d), dtype=np.float32)
    lab = rng.integers(0, b, n)
    x = (c[lab] + sigma * rng.standard_normal((n, d), dtype=np.float32)).astype(np.float32)
    ql = rng.integers(0, b, nq)
    q = (c[ql] + sigma * rng.standard_normal((nq, d), dtype=np.float32)).astype(np.float32)
    if ints:  # small integers: many exactly tied distances at the k-th score
        x, q = np.round(x).astype(np.float32), np.round(q).astype(np.float32)
    d2b = lab.astype(np.int32)[:, None]
    cd = oracle.centroid_dist(q, c)
    probe = oracle.probe_nearest(cd, nprobe)
    return x, q, d2b, probe


@pytest.mark.parametrize("d,k,nq,ints", [(16, 10, 600, False), (100, 1, 600, False), (128, 10, 40, True),
                                          (960, 100, 64, False), (33, 65, 300, True)])
def test_early_abandon_exact(d, k, nq, ints):
    # L2 early abandon (partial sums are monotone, so a pair past its row's
    # threshold is dropped): identical to the unpruned scan and to the oracle,
    # including exact ties at the k-th score (integer data), per-partition lists
    # and both probe-ordering schedules (nq >= / < 32 queries per partition)
    b = 8
    x, q, d2b, probe = clustered_case(500 + d, 12000, d, b, nq, 4, ints=ints)
    idx = check_vs_oracle(x, q, d2b, probe, b, k, "L2")
    Dp, Ip, _ = run(idx, q, probe, k)
    Dn, In, _ = run(idx, q, probe, k, prune=False)
    assert np.array_equal(Ip, In) and np.array_equal(bits(Dp), bits(Dn))
    Dp, Ip, _ = run(idx, q, probe, k, per_partition=True, dedup=False)
    Dn, In, _ = run(idx, q, probe, k, per_partition=True, dedup=False, prune=False)
    assert np.array_equal(Ip, In) and np.array_equal(bits(Dp), bits(Dn))
    off, ids = oracle.build_csr(d2b, b)
    Dq, Iq = oracle.scan_per_partition(q, off, ids, oracle.gather_lists(x, off, ids), probe, k, oracle.L2)
    assert np.array_equal(Ip, Iq) and np.array_equal(bits(Dp), bits(Dq))


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
@pytest.mark.parametrize("k", [24, 25, 56, 57, 120, 121, 248, 249])
def test_screen_list_size_boundaries(metric, k):
    # screened path: K2 = 32*RL >= k+8 list keys per row (RL 1/2/4/8, 64 or 32
    # queries per item); k = 249 falls back to the all-exact kernel
    x, q, d2b, probe = random_case(700 + k, 9000, 40, 10, 150, 4, metric, red=0.1)
    check_vs_oracle(x, q, d2b, probe, 10, k, metric)


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
def test_screen_large_norms_and_ties(metric):
    # SIFT-like integer vectors (norms ~ 500, many exactly tied distances): the
    # screening error bound scales with (|q| + R)^2 and must still admit every
    # tied candidate at the k-th score
    rng = np.random.default_rng(31)
    n, d, b = 20000, 128, 16
    c = rng.integers(0, 120, (b, d)).astype(np.float32)
    lab = rng.integers(0, b, n)
    x = np.clip(c[lab] + rng.integers(-6, 7, (n, d)), 0, 255).astype(np.float32)
    q = np.clip(c[rng.integers(0, b, 200)] + rng.integers(-6, 7, (200, d)), 0, 255).astype(np.float32)
    d2b = lab.astype(np.int32)[:, None]
    probe = oracle.probe_nearest(oracle.centroid_dist(q, c), 3)
    for k in (1, 10, 100):
        check_vs_oracle(x, q, d2b, probe, b, k, metric)
        check_vs_oracle(x, q, d2b, probe, b, k, metric, dedup=False)


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
def test_screen_duplicate_rows_force_exact_rescan(metric):
    # 400 exact copies of a few vectors: more candidates tie within the error
    # band of the k-th than a row's screened list holds, so the merge must
    # re-scan those chunks exactly (lira_index_stats_read()[6] counts it)
    rng = np.random.default_rng(41)
    d, b = 24, 4
    base = rng.standard_normal((8, d), dtype=np.float32)
    # copies stored contiguously, so one 256-candidate chunk holds ~100 of them
    x = np.concatenate([np.repeat(base, 400, axis=0), rng.standard_normal((6000, d), dtype=np.float32)])
    d2b = rng.integers(0, b, (x.shape[0], 1)).astype(np.int32)
    q = np.concatenate([base, rng.standard_normal((40, d), dtype=np.float32)]).astype(np.float32)
    probe = np.tile(np.arange(b, dtype=np.int32), (q.shape[0], 1))
    check_vs_oracle(x, q, d2b, probe, b, 10, metric)
    idx2 = check_vs_oracle(x, q, d2b, probe, b, 10, metric, dedup=False)
    # (k_screen_m: k_screen_r, the L2 default, spills its full lists' evicted keys instead;
    # with no spill list (0) or one that overflows (1 record) it re-scans them too)
    D_, I_, _ = run(idx2, q, probe, 10, dedup=False)
    for sp in (0, 1):
        idx2.set_option("spill", sp)
        D2, I2, _ = run(idx2, q, probe, 10, dedup=False)
        assert np.array_equal(I2, I_) and np.array_equal(bits(D2), bits(D_)), ("spill", sp)
    idx2.set_option("spill", -1)
    idx2.set_option("rscreen", 0)
    idx2.set_stats(True)
    run(idx2, q, probe, 10, dedup=False)
    st = idx2.stats_read()
    idx2.set_stats(False)
    assert st["rescans"] > 0
    # the same re-scans through k_rescan: same results, same count
    idx2.set_option("rescan", 1)
    idx2.set_stats(True)
    D1, I1, _ = run(idx2, q, probe, 10, dedup=False)
    st1 = idx2.stats_read()
    idx2.set_stats(False)
    idx2.set_option("rescan", 0)
    D0, I0, _ = run(idx2, q, probe, 10, dedup=False)
    assert st1["rescans"] == st["rescans"]
    assert np.array_equal(I1, I0) and np.array_equal(bits(D1), bits(D0))
    off, ids = oracle.build_csr(d2b, b)
    met = oracle.IP if metric == "inner_product" else oracle.L2
    Dq, Iq = oracle.scan_per_partition(q, off, ids, oracle.gather_lists(x, off, ids), probe, 10, met)
    D, I, _ = run(idx2, q, probe, 10, per_partition=True, dedup=False)
    assert np.array_equal(I, Iq) and np.array_equal(bits(D), bits(Dq))


def test_compact_index_refuses_tile_paths():
    from lira_amd import LiraError
    x, q, d2b, probe = random_case(11, 3000, 24, 6, 20, 3, "L2")
    idc = make_index(x, d2b, 6, "L2", keep_tiles=False)
    assert idc.get_option("keep_tiles") == 0
    for kw in ({"exact": True}, {"fma": True}):
        with pytest.raises(LiraError, match="EUNSUPPORTED"):
            run(idc, q, probe, 10, **kw)
    with pytest.raises(LiraError, match="EUNSUPPORTED"):
        run(idc, q, probe, 121)
    idc.set_profiling(True)  # a refused call leaves no half-recorded events behind
    with pytest.raises(LiraError):
        run(idc, q, probe, 10, exact=True)
    run(idc, q, probe, 10)
    assert idc.profile_read()["calls"] == 1
    with pytest.raises(LiraError, match="EINVAL"):
        idc.set_option("qr", 96)
    # timing experiments that invalidate results exist only in -DLIRA_DEBUG builds
    idc.set_option("debug", 0)
    with pytest.raises(LiraError, match="EUNSUPPORTED"):
        idc.set_option("debug", 1)


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
def test_options_do_not_change_results(metric):
    x, q, d2b, probe = clustered_case(61, 20000, 48, 8, 700, 3)
    idx = make_index(x, d2b, 8, metric)
    ref = run(idx, q, probe, 10)
    for name, vals in (("qr", (128,)), ("two_phase", (0, 2)), ("seed", (0,)), ("share", (0,)),
                       ("prune", (0,)), ("split", (0,)), ("mfma", (0, 2)), ("rounds", (1, 64)),
                       ("near_rounds", (2, 8)), ("screen", (0,)), ("probes_hint", (1, 4)), ("xhi", (0, 1, 2)),
                       ("rscreen", (0,)), ("rescan", (0, 1)), ("spill", (0, 1, 4)), ("near_first", (0, 1, 4)),
                       ("seed_tiles", (1, 2, 4))):
        old = idx.get_option(name)
        for v in vals:
            idx.set_option(name, v)
            D, I, nc = run(idx, q, probe, 10)
            assert np.array_equal(I, ref[1]) and np.array_equal(bits(D), bits(ref[0])), (name, v)
        idx.set_option(name, old)
    # the build-time storage order (radius-ordered lists vs list order)
    for k in (10, 100):
        idx0 = make_index(x, d2b, 8, metric, order=0)
        D0, I0, _ = run(idx0, q, probe, k)
        D1, I1, _ = run(idx, q, probe, k)
        assert np.array_equal(I0, I1) and np.array_equal(bits(D0), bits(D1)), ("order", k)
        idx.set_option("qr", 32)  # 32 queries per item at RL 4 (k > 56, full split)
        D3, I3, _ = run(idx, q, probe, k)
        idx.set_option("qr", 0)
        assert np.array_equal(I3, I1) and np.array_equal(bits(D3), bits(D1)), ("qr32", k)
    # IP: the uncentred split copy (LIRA_OPT_IP_CENTRE = 0, round 4's layout, k_screen_m)
    if metric == "inner_product":
        idu = make_index(x, d2b, 8, metric, ip_centre=0)
        for k in (10, 100):
            D0, I0, _ = run(idu, q, probe, k)
            D1, I1, _ = run(idx, q, probe, k)
            assert np.array_equal(I0, I1) and np.array_equal(bits(D0), bits(D1)), ("ip_centre", k)
        # an index built uncentred has no fused seed, whatever ip_centre says afterwards
        from lira_amd import LiraError
        idu.set_option("ip_centre", 1)
        with pytest.raises(LiraError, match="EUNSUPPORTED"):
            idu.set_option("seed_tiles", 4)
    # the removed screen variants (k_screen_s / _w / _v, k_seed_b): 0 still reads back, others refused
    from lira_amd import LiraError
    # (4 seed tiles exist only in the fused seeds: refused where neither can run)
    wide = make_index(np.zeros((64, 300), np.float32), np.zeros((64, 1), np.int32), 1, metric)
    with pytest.raises(LiraError, match="EUNSUPPORTED"):
        wide.set_option("seed_tiles", 4)
    for name, bad in (("pipeline", 1), ("ring", 3), ("wide", 1), ("seed", 2)):
        with pytest.raises(LiraError, match="EUNSUPPORTED"):
            idx.set_option(name, bad)
    for name in ("pipeline", "ring", "wide"):
        idx.set_option(name, 0)
        assert idx.get_option(name) == 0


@pytest.mark.parametrize("metric", ["L2", "inner_product"])
def test_split_screen_extreme_values(metric):
    # split-bf16 parts of values near FLT_MAX (the hi part saturates to the
    # largest finite bf16 instead of rounding to infinity) and of subnormals
    rng = np.random.default_rng(71)
    n, d, b = 4000, 16, 4
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((40, d)).astype(np.float32)
    if metric == "inner_product":
        big = rng.random(n) < 0.05
        x[big, 3] = np.float32(3.399e38) * np.sign(rng.standard_normal(big.sum())).astype(np.float32)
        q *= np.float32(1e-3)
    tiny = rng.random(n) < 0.05
    x[tiny] *= np.float32(1e-40)
    q[:5] *= np.float32(1e-39)
    d2b = rng.integers(0, b, (n, 1)).astype(np.int32)
    probe = np.tile(np.arange(b, dtype=np.int32), (q.shape[0], 1))
    check_vs_oracle(x, q, d2b, probe, b, 10, metric)


@pytest.mark.parametrize("d,uniform,red", [(48, False, 0.0), (96, False, 0.2), (128, False, 0.0), (128, True, 0.0),
                                           (100, True, 0.1)])
def test_screen_many_blocks_vs_oracle(d, uniform, red):
    # the default screen over several query blocks per list, lists of several
    # chunks with a partial last block (one tile) and padded rows, partial query
    # blocks, redundant rows with and without dedup, at 1 / 8 (auto) / 64 items
    # per workgroup
    n, b, nq, nprobe, k = 60000, 10, 1500, 4, 10
    x, q, d2b, probe = random_case(300 + d, n, d, b, nq, nprobe, "L2", red=red, uniform=uniform)
    idx = make_index(x, d2b, b, "L2")
    off, ids = oracle.build_csr(d2b, b)
    vecs = oracle.gather_lists(x, off, ids)
    for dedup in (True, False):
        Do, Io, nco = oracle.scan_topk(q, off, ids, vecs, probe, k, oracle.L2, idx.max_replicas if dedup else 0)
        for rounds in (0, 1, 64):  # items of whole lists, and many short chunks
            idx.set_option("rounds", rounds)
            D, I, nc = run(idx, q, probe, k, dedup=dedup)
            assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do)), (dedup, rounds)
            assert np.array_equal(nc, nco)
        idx.set_option("rounds", 0)


def test_screen_clustered_filter_and_ties():
    # separated clusters: the plan's filter drops the far pairs (no work items,
    # counted), the triangle skip drops blocks; small-integer vectors: exact
    # ties at the k-th
    x, q, d2b, probe = clustered_case(71, 40000, 128, 16, 900, 6, ints=True)
    idx = make_index(x, d2b, 16, "L2")
    off, ids = oracle.build_csr(d2b, 16)
    vecs = oracle.gather_lists(x, off, ids)
    for k in (1, 10, 24):
        Do, Io, nco = oracle.scan_topk(q, off, ids, vecs, probe, k, oracle.L2, idx.max_replicas)
        D, I, nc = run(idx, q, probe, k)
        assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do)), k
        assert np.array_equal(nc, nco)
        idx.set_stats(True)
        run(idx, q, probe, k)
        st = idx.stats_read()
        idx.set_stats(False)
        assert st["blocks"] > 0
        assert st["pairs_pruned_plan"] > 0 and st["candidates_pruned_plan"] >= st["pairs_pruned_plan"]


def test_graph_replay_after_eager_calls():
    # a captured step replayed after eager calls of the same search (the per-call
    # resets are a kernel of the library's own, not hipMemsetAsync: a captured memset
    # replayed after an eager one faulted, lira_device.hpp fill32_async)
    import torch
    from lira_amd import PartitionedIndex, rank_nearest
    dev = torch.device("cuda", 0)
    x, q, d2b, probe = random_case(91, 20000, 32, 16, 500, 4, "L2")
    c = torch.from_numpy(np.stack([x[d2b[:, 0] == b].mean(0) for b in range(16)]).astype(np.float32)).to(dev)
    xt, qt = torch.from_numpy(x).to(dev), torch.from_numpy(q).to(dev)
    for keep in (True, False):
        idx = PartitionedIndex(32, "L2", 0, keep_tiles=int(keep)).build(torch.from_numpy(d2b).to(dev), xt, 16)
        pr = torch.empty((500, 4), dtype=torch.int32, device=dev)
        D = torch.empty((500, 10), dtype=torch.float32, device=dev)
        I = torch.empty((500, 10), dtype=torch.int64, device=dev)
        nc = torch.empty(500, dtype=torch.int64, device=dev)

        def step():
            rank_nearest(qt, c, 4, out=pr)
            idx.search(qt, pr, 10, out=(D, I, nc))

        step()
        step()
        torch.cuda.synchronize()
        I0, D0 = I.clone(), D.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        for _ in range(3):
            g.replay()
        for prof in (False, True):
            idx.set_profiling(prof)
            for _ in range(3):
                step()
            idx.set_profiling(False)
            I.zero_()
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(I, I0) and torch.equal(D.view(torch.int32), D0.view(torch.int32)), (keep, prof)
        del g


def unit_case(seed, n, d, b, nq, nprobe, sigma=0.5):
    # L2-normalised rows around b random directions (DEEP1B-like: search.cpp's IP on unit vectors)
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((b, d), dtype=np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    lab = rng.integers(0, b, n)
    x = c[lab] + sigma / np.sqrt(d) * rng.standard_normal((n, d), dtype=np.float32)
    x = (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)
    q = c[rng.integers(0, b, nq)] + sigma / np.sqrt(d) * rng.standard_normal((nq, d), dtype=np.float32)
    q = (q / np.linalg.norm(q, axis=1, keepdims=True)).astype(np.float32)
    d2b = oracle.centroid_dist(x, c).argmin(1).astype(np.int32)[:, None]
    probe = oracle.probe_nearest(oracle.centroid_dist(q, c), nprobe)
    return x, q, d2b, probe


@pytest.mark.parametrize("k", [10, 40, 100])
@pytest.mark.parametrize("data", ["clustered", "unit"])
def test_rscreen_ip_centred(k, data):
    # k_screen_r on a centred IP index (q.x = q.fl(x - c) + q.c, Cauchy-Schwarz block
    # skip and plan filter; 32-, 64- and 128-key row lists): bit-exact against the
    # oracle, the uncentred index (LIRA_OPT_IP_CENTRE = 0: k_screen_m) and the options
    n, d, b, nq, nprobe = 40000, 96, 16, 700, 5
    if data == "clustered":
        x, q, d2b, probe = clustered_case(800 + k, n, d, b, nq, nprobe)
    else:
        x, q, d2b, probe = unit_case(900 + k, n, d, b, nq, nprobe)
    idx = make_index(x, d2b, b, "inner_product")
    assert idx.describe(nq, nprobe, k).startswith("k_screen_r"), idx.describe(nq, nprobe, k)
    off, ids = oracle.build_csr(d2b, b)
    vecs = oracle.gather_lists(x, off, ids)
    for dedup in (True, False):
        Do, Io, nco = oracle.scan_topk(q, off, ids, vecs, probe, k, oracle.IP, idx.max_replicas if dedup else 0)
        D, I, nc = run(idx, q, probe, k, dedup=dedup)
        assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do)), dedup
        assert np.array_equal(nc, nco)
    idx.set_stats(True)
    run(idx, q, probe, k)
    st = idx.stats_read()
    idx.set_stats(False)
    assert st["survivors"] > 0
    if data == "clustered":  # far clusters: whole lists or tiles dropped by Cauchy-Schwarz
        assert st["blocks_skipped"] + st["pairs_pruned_plan"] > 0, st
    ref = run(idx, q, probe, k)
    for name, v in (("spill", 0), ("spill", 1), ("near_first", 0), ("rescan", 1), ("prune", 0), ("rounds", 64),
                    ("qr", 64)):  # (qr 64 at k > 24: 8 waves per item of 64 rows)
        old = idx.get_option(name)
        idx.set_option(name, v)
        D, I, _ = run(idx, q, probe, k)
        idx.set_option(name, old)
        assert np.array_equal(I, ref[1]) and np.array_equal(bits(D), bits(ref[0])), (name, v)
    idu = make_index(x, d2b, b, "inner_product", ip_centre=0)
    assert not idu.describe(nq, nprobe, k).startswith("k_screen_r")
    D, I, _ = run(idu, q, probe, k)
    assert np.array_equal(I, ref[1]) and np.array_equal(bits(D), bits(ref[0])), "uncentred"
    # per-partition lists on the centred index run the fp32-tile screen
    Dp, Ip, _ = run(idx, q, probe, k, per_partition=True, dedup=False)
    Dq, Iq = oracle.scan_per_partition(q, off, ids, vecs, probe, k, oracle.IP)
    assert np.array_equal(Ip, Iq) and np.array_equal(bits(Dp), bits(Dq))


@pytest.mark.parametrize("k", [25, 64, 100])
def test_rscreen_l2_long_lists(k):
    # L2 at k > 24: k_screen_r with 32 query rows per item and 64 / 128-key row lists
    x, q, d2b, probe = clustered_case(1000 + k, 40000, 64, 16, 700, 5, spread=0.6)
    idx = make_index(x, d2b, 16, "L2")
    assert idx.describe(700, 5, k).startswith("k_screen_r")
    off, ids = oracle.build_csr(d2b, 16)
    Do, Io, nco = oracle.scan_topk(q, off, ids, oracle.gather_lists(x, off, ids), probe, k, oracle.L2,
                                   idx.max_replicas)
    D, I, nc = run(idx, q, probe, k)
    assert np.array_equal(I, Io) and np.array_equal(bits(D), bits(Do))
    idx.set_option("rscreen", 0)
    D2, I2, _ = run(idx, q, probe, k)
    assert np.array_equal(I2, Io) and np.array_equal(bits(D2), bits(Do))


def test_graph_capture_workspace_growth():
    # the handle's cached workspace (lira_hip.h lira_scan_topk): growing it while the
    # stream is captured is refused (EINVAL); an eager call that outgrows a buffer a
    # captured graph uses leaves that buffer allocated, so the replay stays valid
    import torch
    from lira_amd import LiraError
    dev = torch.device("cuda", 0)
    x, q, d2b, probe = random_case(93, 20000, 32, 16, 3000, 4, "L2")
    qt, pt = torch.from_numpy(q).to(dev), torch.from_numpy(probe).to(dev)
    idx = make_index(x, d2b, 16, "L2")
    D = torch.empty((200, 10), dtype=torch.float32, device=dev)
    I = torch.empty((200, 10), dtype=torch.int64, device=dev)
    nc = torch.empty(200, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        idx.search(qt[:200], pt[:200], 10, out=(D, I, nc))  # sizes the cached workspace
        torch.cuda.synchronize()
        I0, D0 = I.clone(), D.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            idx.search(qt[:200], pt[:200], 10, out=(D, I, nc))
        run(idx, q, probe, 10)  # 3000 queries: a larger workspace (the captured one retired)
        I.zero_()
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(I, I0) and torch.equal(D.view(torch.int32), D0.view(torch.int32))
    del g
    # a fresh handle: its first call would allocate under capture
    idx2 = make_index(x, d2b, 16, "L2")
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with pytest.raises(LiraError, match="EINVAL"):
            with torch.cuda.graph(g2, stream=s):
                idx2.search(qt[:200], pt[:200], 10, out=(D, I, nc))
    torch.cuda.synchronize()
    del g2


def test_two_streams_one_handle():
    # lira_hip.h "Threading and streams": two torch streams search ONE handle at the
    # same time with the cached workspace (workspace = NULL); each stream gets its own
    # buffer, so both results equal the oracle's.  Then the 8-stream cap: 8 streams
    # whose buffers captured graphs pin, a 9th eager stream is refused (ESTATE).
    import torch
    from lira_amd import LiraError
    dev = torch.device("cuda", 0)
    x, q, d2b, probe = clustered_case(97, 30000, 64, 16, 1500, 4)
    idx = make_index(x, d2b, 16, "L2")
    off, ids = oracle.build_csr(d2b, 16)
    vecs = oracle.gather_lists(x, off, ids)
    halves = [(0, 900), (900, 1500)]  # different sizes: different plans and workspaces
    want = [oracle.scan_topk(q[a:b], off, ids, vecs, probe[a:b], 10, oracle.L2, 1) for a, b in halves]
    qt, pt = torch.from_numpy(q).to(dev), torch.from_numpy(probe).to(dev)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [(torch.empty((b - a, 10), dtype=torch.float32, device=dev),
             torch.empty((b - a, 10), dtype=torch.int64, device=dev),
             torch.empty(b - a, dtype=torch.int64, device=dev)) for a, b in halves]
    torch.cuda.synchronize()
    for rep in range(4):
        for s, (a, b), o in zip(streams, halves, outs):  # enqueued back to back, no sync between
            with torch.cuda.stream(s):
                o[1].fill_(-7)
                idx.search(qt[a:b], pt[a:b], 10, out=o)
        torch.cuda.synchronize()
        idx.check()
        for (Do, Io, nco), (D, I, nc) in zip(want, outs):
            assert np.array_equal(I.cpu().numpy(), Io), rep
            assert np.array_equal(bits(D.cpu().numpy()), bits(Do)), rep
            assert np.array_equal(nc.cpu().numpy(), nco), rep
    # 8 streams whose buffers are held by captured graphs: a 9th stream cannot take one
    graphs, gs = [], [torch.cuda.Stream() for _ in range(8)]
    D, I, nc = outs[0]
    for s in gs:
        with torch.cuda.stream(s):
            idx.search(qt[:900], pt[:900], 10, out=(D, I, nc))  # sizes this stream's buffer
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                idx.search(qt[:900], pt[:900], 10, out=(D, I, nc))
            graphs.append(g)
    torch.cuda.synchronize()
    s9 = torch.cuda.Stream()
    with torch.cuda.stream(s9):
        with pytest.raises(LiraError, match="ESTATE"):
            idx.search(qt[:900], pt[:900], 10, out=(D, I, nc))
        # ... while a caller-supplied workspace always works
        ws = torch.empty(idx.workspace_size(900, 4, 10), dtype=torch.uint8, device=dev)
        idx.search(qt[:900], pt[:900], 10, out=(D, I, nc), workspace=ws)
    torch.cuda.synchronize()
    assert np.array_equal(I.cpu().numpy(), want[0][1])
    graphs[3].replay()
    torch.cuda.synchronize()
    assert np.array_equal(I.cpu().numpy(), want[0][1])
    del graphs
