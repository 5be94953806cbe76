"""CPU model check of k_screen_r's screening error bounds (lira_rscreen.hip errE_r):
the screened score of the hi x hi split-bf16 screen on the centred copy must lie
within E of search.cpp's exact fp32 score (search.cpp:253-269: sequential sums of
rounded terms, no FMA) for every candidate.  The screen's MFMA sum is modelled as a
sequential fp32 sum (the bound's accumulation term allows any order); the rest is
the kernel's own arithmetic.  No GPU: numpy float32 emulation."""
import numpy as np
import pytest

U = 2.0 ** -24


def bf16_hi(v):
    b = np.ascontiguousarray(v, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def seq_sum(terms):
    acc = np.zeros(terms.shape[0], dtype=np.float32)
    for j in range(terms.shape[1]):
        acc = (acc + terms[:, j]).astype(np.float32)
    return acc


def err_ip(qnorm, Rb, hres, qres, dp, qc, Rx, d):
    # lira_rscreen.hip errE_r<IP> (double here: the kernel rounds it up in fp32)
    ex = hres * 1.0001
    ed = (ex * qnorm + qres * (Rb + ex) * 1.0001 + 2.0 * (dp + 1.0) * 2.0 ** -22 * 1.02 * qnorm * (Rb + ex)
          + 2.0 * dp * 2.0 ** -96 * (qnorm + Rb + ex + 1.0))
    aq = abs(qc)
    return (ed + (1.01 * qnorm * Rb + 2.02 * aq + qnorm * (Rb + ex) + (d + 2.0) * qnorm * Rx) * U) * 1.05


def err_l2(qnorm, Rb, hres, qres, dp):
    ex = hres * 1.0001
    ed = (ex * qnorm + qres * (Rb + ex) * 1.0001
          + 2.0 * (dp + 1.0) * 2.0 ** -22 * 1.02 * (qnorm * (Rb + ex) + 0.5001 * Rb * Rb)
          + 2.0 * dp * 2.0 ** -96 * (qnorm + Rb + ex + 1.0))
    s = qnorm + Rb
    return 2.0 * ed + (1.05 * 8.0 + 2.01 + 2.0) * U * s * s


@pytest.mark.parametrize("seed,d,scale,offset", [(1, 96, 1.0, 0.0), (2, 96, 1.0, 3.0), (3, 128, 30.0, 0.0),
                                                   (4, 32, 1e-3, 5e-3), (5, 960, 1.0, 0.5), (6, 96, 1.0, -2.0)])
def test_ip_centred_bound(seed, d, scale, offset):
    rng = np.random.default_rng(seed)
    n = 4000
    c = (offset + rng.standard_normal(d)).astype(np.float32) * np.float32(scale)
    x = (c + np.float32(scale) * 0.4 * rng.standard_normal((n, d))).astype(np.float32)
    q = (np.float32(scale) * rng.standard_normal(d)).astype(np.float32)
    piv = x.mean(0, dtype=np.float64).astype(np.float32)
    xc = (x - piv).astype(np.float32)  # fl(x - c), the split copy's values
    xh, qh = bf16_hi(xc), bf16_hi(q)
    dp = float((d + 31) // 32 * 32)
    qnorm = float(np.sqrt((q.astype(np.float64) ** 2).sum())) * (1 + 2 ** -40)
    qres = float(np.sqrt(((q - qh).astype(np.float64) ** 2).sum())) * (1 + 2 ** -40)
    hres = float(np.sqrt(((xc - xh).astype(np.float64) ** 2).sum(1)).max()) * (1 + 2 ** -40)
    Rb = float(np.sqrt((xc.astype(np.float64) ** 2).sum(1)).max()) * (1 + 2 ** -20)
    Rx = float(np.sqrt((x.astype(np.float64) ** 2).sum(1)).max()) * (1 + 2 ** -40)
    qc = float(np.dot(q.astype(np.float64), piv.astype(np.float64)))
    qcf = np.float32(qc)
    wv = seq_sum((qh[None, :] * xh).astype(np.float32))  # products of bf16 parts are exact in fp32
    s_scr = -(wv + qcf).astype(np.float32)
    s_ex = -seq_sum((q[None, :] * x).astype(np.float32))  # search.cpp ip, ranked as -ip
    E = err_ip(qnorm, Rb, hres, qres, dp, qc, Rx, d)
    gap = np.abs(s_scr.astype(np.float64) - s_ex.astype(np.float64))
    assert gap.max() <= E, (gap.max(), E)
    assert E < 0.05 * (np.abs(s_ex).max() + 1e-30) or scale < 1e-2  # the bound is not vacuous


@pytest.mark.parametrize("seed,d,scale", [(11, 128, 1.0), (12, 128, 100.0), (13, 96, 1.0)])
def test_l2_centred_bound(seed, d, scale):
    rng = np.random.default_rng(seed)
    n = 4000
    c = (rng.standard_normal(d) * scale).astype(np.float32)
    x = (c + scale * 0.4 * rng.standard_normal((n, d))).astype(np.float32)
    q = (c + scale * 0.4 * rng.standard_normal(d)).astype(np.float32)
    piv = x.mean(0, dtype=np.float64).astype(np.float32)
    xc, qcen = (x - piv).astype(np.float32), (q - piv).astype(np.float32)
    xh, qh = bf16_hi(xc), bf16_hi(qcen)
    dp = float((d + 31) // 32 * 32)
    qnorm = float(np.sqrt((qcen.astype(np.float64) ** 2).sum())) * (1 + 2 ** -40)
    qres = float(np.sqrt(((qcen - qh).astype(np.float64) ** 2).sum())) * (1 + 2 ** -40)
    hres = float(np.sqrt(((xc - xh).astype(np.float64) ** 2).sum(1)).max()) * (1 + 2 ** -40)
    Rb = float(np.sqrt((xc.astype(np.float64) ** 2).sum(1)).max()) * (1 + 2 ** -20)
    xadj = (np.float32(0.5) * ((xc.astype(np.float64) ** 2).sum(1)).astype(np.float32)).astype(np.float32)
    qn = np.float32((qcen.astype(np.float64) ** 2).sum())
    acc = seq_sum(np.concatenate([-xadj[:, None], (qh[None, :] * xh).astype(np.float32)], axis=1))
    s_scr = (qn - np.float32(2.0) * acc).astype(np.float32)
    s_ex = seq_sum(((q[None, :] - x) ** 2).astype(np.float32))  # search.cpp l2_sq
    g = (d + 4.0) * U  # search.cpp's own rounding: bound_P / s_lim carry (1 +- g)
    E = err_l2(qnorm, Rb, hres, qres, dp)
    lo = s_ex.astype(np.float64) * (1 - g) - d * 2.0 ** -140 - E
    hi = s_ex.astype(np.float64) * (1 + g) + d * 2.0 ** -140 + E
    # (the screen's s~ vs the real D = ||q - x||^2 within E, and search.cpp's s within g of D)
    D = ((q.astype(np.float64) - x.astype(np.float64)) ** 2).sum(1)
    assert (np.abs(s_scr - D) <= E).all()
    assert ((s_scr >= lo) & (s_scr <= hi)).all()
