"""CPU: the oracle (oracle/lira_oracle.c, the parity checker) built with
AddressSanitizer + UBSan (`make -C oracle sanitize`) and run on every golden
fixture and on edge cases (empty buckets, k above the candidate count, -1 and
duplicate probe slots, redundancy without dedup, d = 1): it must finish clean and
give the fixtures' expected outputs bit for bit, as tests/test_oracle.py checks
for the normal build -- so an out-of-bounds access in the checker cannot mask a
parity failure."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import load_golden

HERE = os.path.dirname(os.path.abspath(__file__))
ODIR = os.path.join(os.path.dirname(HERE), "oracle")
DRIVER = os.path.join(ODIR, "build", "sanitize_driver")


@pytest.fixture(scope="module")
def driver():
    subprocess.run(["make", "-s", "-C", ODIR, "sanitize"], check=True)
    return DRIVER


def run_case(driver, tmp_path, x, d2b, q, probe, cent, mean, scale, k, metric, rep):
    n, d = x.shape
    nq, np_ = probe.shape
    nb = cent.shape[0]
    case, out = tmp_path / "case.bin", tmp_path / "out.bin"
    with open(case, "wb") as f:
        f.write(np.array([n, d, d2b.shape[1], nb, nq, np_, k, metric, rep], np.int64).tobytes())
        for a, t in ((x, np.float32), (d2b, np.int32), (q, np.float32), (probe, np.int32), (cent, np.float32),
                     (mean, np.float32), (scale, np.float32)):
            f.write(np.ascontiguousarray(a, t).tobytes())
    env = dict(os.environ, OMP_NUM_THREADS="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([driver, str(case), str(out)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    buf = open(out, "rb").read()
    pos = 0

    def take(dtype, count):
        nonlocal pos
        a = np.frombuffer(buf, dtype, count, pos)
        pos += a.nbytes
        return a

    total = int(take(np.int64, 1)[0])
    res = {"offsets": take(np.int64, nb + 1), "ids": take(np.int32, total),
           "D": take(np.float32, nq * k).reshape(nq, k), "I": take(np.int64, nq * k).reshape(nq, k),
           "ncand": take(np.int64, nq),
           "D_part": take(np.float32, nq * np_ * k).reshape(nq, np_, k),
           "I_part": take(np.int64, nq * np_ * k).reshape(nq, np_, k),
           "qdist": take(np.float32, nq * nb).reshape(nq, nb), "qdist_std": take(np.float32, nq * nb).reshape(nq, nb),
           "probe_nearest": take(np.int32, nq * np_).reshape(nq, np_),
           "probe_ge": take(np.int32, nq * nb).reshape(nq, nb), "count_ge": take(np.int32, nq),
           "probe_gt": take(np.int32, nq * nb).reshape(nq, nb), "count_gt": take(np.int32, nq)}
    assert pos == len(buf)
    return res


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float32).view(np.uint32),
                          np.ascontiguousarray(b, np.float32).view(np.uint32))


def check_selects(r, nprobe):
    # the selections against the unsanitized library on the same (bit-equal) inputs
    assert np.array_equal(r["probe_nearest"], oracle.probe_nearest(r["qdist"], nprobe))
    for strict, key in ((False, "ge"), (True, "gt")):
        p, c = oracle.probe_threshold(r["qdist_std"], 0.0, strict=strict)
        assert np.array_equal(r["probe_" + key], p) and np.array_equal(r["count_" + key], c)


@pytest.mark.parametrize("name", ["toy_l2", "toy_ip", "sift_like_redundant", "deep_like_k100_ip", "odd_dim"])
def test_sanitized_oracle_reproduces_golden(driver, tmp_path, name):
    g = load_golden(name)
    met = oracle.IP if str(g["metric"]) == "inner_product" else oracle.L2
    r = run_case(driver, tmp_path, g["x"], g["data_2_bkt"], g["q"], g["probe"], g["centroids"], g["scaler_mean"],
                 g["scaler_scale"], int(g["k"]), met, int(g["dedup_rep"]))
    assert np.array_equal(r["offsets"], g["offsets"]) and np.array_equal(r["ids"], g["ids"])
    assert same_bits(r["D"], g["D"]) and np.array_equal(r["I"], g["I"]) and np.array_equal(r["ncand"], g["ncand"])
    assert same_bits(r["D_part"], g["D_part"]) and np.array_equal(r["I_part"], g["I_part"])
    assert same_bits(r["qdist"], g["qdist"]) and same_bits(r["qdist_std"], g["qdist_std"])
    check_selects(r, g["probe"].shape[1])


@pytest.mark.parametrize("metric", [oracle.L2, oracle.IP])
@pytest.mark.parametrize("rep", [0, 2])
def test_sanitized_oracle_edge_cases(driver, tmp_path, metric, rep):
    rng = np.random.default_rng(40 + metric + rep)
    for n, d, nb, nq, nprobe, k in ((300, 1, 7, 9, 4, 50), (500, 13, 9, 17, 9, 3), (40, 5, 6, 3, 6, 64)):
        x = rng.standard_normal((n, d), dtype=np.float32)
        q = rng.standard_normal((nq, d), dtype=np.float32)
        cent = rng.standard_normal((nb, d), dtype=np.float32)
        d2b = np.full((n, 2), -1, np.int32)
        d2b[:, 0] = rng.integers(0, nb - 2, n)  # the last two buckets stay empty
        red = rng.random(n) < 0.3
        d2b[red, 1] = rng.integers(0, nb, red.sum())
        dup = red & (rng.random(n) < 0.2)
        d2b[dup, 1] = d2b[dup, 0]  # the same bucket twice in one row (search.cpp:381-385 collapses it)
        probe = rng.integers(-1, nb, (nq, nprobe)).astype(np.int32)  # -1 slots, repeats, empty buckets
        probe[0, :] = -1  # a query that probes nothing
        mean = rng.standard_normal(nb).astype(np.float32)
        scale = rng.random(nb).astype(np.float32)
        scale[1] = 0.0  # search.cpp:247: scale 0 -> 1
        r = run_case(driver, tmp_path, x, d2b, q, probe, cent, mean, scale, k, metric, rep)
        off, ids = oracle.build_csr(d2b, nb)
        assert np.array_equal(r["offsets"], off) and np.array_equal(r["ids"], ids)
        vecs = oracle.gather_lists(x, off, ids)
        D, I, nc = oracle.scan_topk(q, off, ids, vecs, probe, k, metric, rep)
        assert same_bits(r["D"], D) and np.array_equal(r["I"], I) and np.array_equal(r["ncand"], nc)
        Dp, Ip = oracle.scan_per_partition(q, off, ids, vecs, probe, k, metric)
        assert same_bits(r["D_part"], Dp) and np.array_equal(r["I_part"], Ip)
        assert same_bits(r["qdist"], oracle.centroid_dist(q, cent))
        assert same_bits(r["qdist_std"], oracle.centroid_dist(q, cent, mean, scale))
        assert (r["I"][0] == -1).all()
        check_selects(r, nprobe)
