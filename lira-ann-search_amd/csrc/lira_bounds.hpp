// lira_bounds.hpp -- the screen's rigorous error model (double precision),
// shared by the screening kernels (lira_screen.hip, lira_wscreen.hip).  The
// derivation is in lira_screen.hip's header and DESIGN.md section 4.3.
#pragma once
#include "lira_device.hpp"

namespace lira {

static constexpr double kU = 0x1p-24;

// ---- error model (double) -------------------------------------------------
// split != 0: the dot product came from the split-bf16 MFMA screen
// (k_screen_m<..., SPLIT>): q = qh + ql + eq, x = xh + xl + ex with every part a
// bf16 round-to-nearest (|eq| <= 2^-16 |q_i|, |ex| <= 2^-16 |x_i|), the four
// exact products qh xh, qh xl, ql xh, ql xl summed in fp32 in an unspecified
// order (4 dpad terms, <= 2^-22 relative per add: any rounding mode the
// matrix core may use), so |dot~ - q.x| <= ed = (2.0001 2^-16 + 4 dpad 2^-22)
// 1.02 |q| R + an absolute term for flushed subnormal parts (values below
// 2^-100 lose at most 2^-100 (|q| + R) per product).  The rest of the L2
// score's error (qn, xn, their sum, the final fma) stays <= 8.4 u (|q|+R)^2.
//
// centred (L2, split screen): q' = fl(q - c), x' = fl(x - c) for the list's
// pivot c, and qnorm, R the norms of q', x'.  Then (q' - x') - (q - x) =
// (q - c) e1 - (x - c) e2 with |e| <= u per component, so ||q'-x'||^2 differs
// from D = ||q-x||^2 by at most u s (2 + u) s (1 + u) <= 2.01 u s^2, s = qnorm
// + R, on top of the screen's own error for q', x'.
//
// split == 3 (hi x hi, k_screen_m<..., 3>): dot~ = sum qh xh, one product per
// dim (exact in fp32), so q.x - dot~ = q.(x - xh) + (q - qh).xh and
// |dot~ - q.x| <= |q| ||ex|| + qres (R + ||ex||) + (2 dpad 2^-22) 1.02 |q| (R +
// ||ex||) + the subnormal term, qres >= ||q - qh|| of the row (k_qstage, QE).
template <int METRIC>
__device__ __forceinline__ double err_E(double qnorm, double R, double d, int split = 0, double dp = 0.0,
                                        int centred = 0, double hres = -1.0, double qres = 0.0) {
    const double dl = d * 0x1p-140;
    if (split == 3) {
        const double ex = hres >= 0.0 ? hres * 1.0001 : 0x1p-8 * 1.02 * R;
        const double ed = ex * qnorm + qres * (R + ex) * 1.0001 + 2.0 * dp * 0x1p-22 * 1.02 * qnorm * (R + ex) +
                          2.0 * dp * 0x1p-96 * (qnorm + R + ex + 1.0);
        if (METRIC == LIRA_METRIC_L2) {
            const double s = qnorm + R;
            return 2.0 * ed + (1.05 * 8.0 + (centred ? 2.01 : 0.0)) * kU * s * s + dl;
        }
        return 1.05 * (ed + (d + 2.0) * kU * qnorm * R) + dl;
    }
    if (split) {
        // split == 2 (hi-only x, k_screen_m<..., 2>): dot~ = sum (qh + ql) xh, x = xh + ex:
        // |dot~ - q.x| <= |q.ex| + |(q - qh - ql).xh| + rounding <= |q| ||ex|| +
        // (2^-16 + 2 dpad 2^-22) 1.02 |q| R, with ||ex|| <= 2^-8 R (|ex_i| <= 2^-8 |x_i|)
        // or, tighter, hres >= ||ex|| of every candidate concerned (lira_abi.hip k_row_stats)
        const double ex = hres >= 0.0 ? hres * 1.0001 : 0x1p-8 * 1.02 * R;
        const double ed = split == 2 ? ex * qnorm + (1.0001 * 0x1p-16 + 2.0 * dp * 0x1p-22) * 1.02 * qnorm * R +
                                           2.0 * dp * 0x1p-96 * (qnorm + R + 1.0)
                                     : (2.0001 * 0x1p-16 + 4.0 * dp * 0x1p-22) * 1.02 * qnorm * R +
                                           4.0 * dp * 0x1p-96 * (qnorm + R + 1.0);
        if (METRIC == LIRA_METRIC_L2) {
            const double s = qnorm + R;
            return 2.0 * ed + (1.05 * 8.0 + (centred ? 2.01 : 0.0)) * kU * s * s + dl;
        }
        // IP: bound_P / s_lim carry no (1 +- g) factor, so E also covers
        // search.cpp's own rounding of the exact sum, (d+2) u |q| R (L2 needs
        // no such term: that error is the g of bound_P / s_lim)
        return 1.05 * (ed + (d + 2.0) * kU * qnorm * R) + dl;
    }
    if (METRIC == LIRA_METRIC_L2) {
        const double s = qnorm + R;
        return 1.05 * ((d + 8.0) * kU * s * s) + dl;
    }
    return 1.05 * (2.0 * (d + 2.0) * kU * qnorm * R) + dl;
}
// bound on the final k-th exact score from a list's k-th screened score
template <int METRIC>
__device__ __forceinline__ double bound_P(double sk, double E, double d) {
    if (METRIC == LIRA_METRIC_L2) return (sk + E) * (1.0 + (d + 4.0) * kU) * (1.0 + 0x1p-50) + d * 0x1p-140;
    return (sk + E) + __builtin_fabs(sk + E) * 0x1p-50;
}
// largest screened score a candidate may have and still score <= T exactly
template <int METRIC>
__device__ __forceinline__ double s_lim(double T, double E, double d) {
    if (METRIC == LIRA_METRIC_L2) return ((T + d * 0x1p-140) / (1.0 - (d + 4.0) * kU)) * (1.0 + 0x1p-50) + E;
    return T + E + __builtin_fabs(T + E) * 0x1p-50;
}
// per-block test threshold on the dot product: pass iff fl(dot - xadj) >= h.
// L2: s~ <= lim  <=>  dot - xn/2 >= (qn - lim)/2; fl(dot - xadj) is off by at
// most u (|q| + R)^2.  IP: xadj = 0, -s~ = dot >= -lim.
template <int METRIC>
__device__ __forceinline__ float row_h(double lim, double qn, double qnorm, double R) {
    if (!(lim < 1e300)) return -__builtin_inff();
    double h;
    if (METRIC == LIRA_METRIC_L2) {
        const double s = qnorm + R;
        h = (qn - lim) * 0.5 - 1.05 * kU * s * s;
    } else {
        h = -lim;
    }
    h -= __builtin_fabs(h) * 0x1p-50;
    return __double2float_rd(h);
}



// ---- per-pair records + the partition filter (k_pairs, k_seed_t<..., PAIRS>) ----
// 16 lanes per (query, slot) pair (sub = lane & 15; all 16 call it), double sums:
// qn = fl(||q'||^2), qnorm >= ||q'||, q' = fl(q - c) of the pair's list pivot c
// (centred) or q; dq = fl(||q - c||) (triangle skip); qres >= ||q' - hi(q')||
// (hi x hi bound); QH (optional): hi(q') as bf16, dpad dims, zero past d (the
// rows' A fragments of k_screen_m / k_screen_v, gathered per pair).
// Filter (lstat, qb = f2ord of the query's seed bound T): a pair whose list
// lies wholly outside the query's triangle interval under T (k exact
// candidates of its slot-0 list score <= T) cannot hold a top-k candidate, so
// it gets probe_live = -1 and no work item (the test is k_screen_m's per-block
// skip over the list's radius range).  Slot 0 (the seed's own list) stays.
// (est_size / est_samp set) returns, in every lane of the pair's 16, an
// estimate of the screen blocks the pair will compute: its whole list for slot
// 0, else the share of 16 evenly spaced tiles of its (radius-ordered) list whose
// radius range meets the query's triangle interval under the seed bound -- the
// plan sizes the nearest-probe group's items from the batch's total (0 for an
// invalid or filtered pair)
//
// centred == 2 (IP on a centred copy, k_screen_r): q is NOT centred (q' = q); the
// record carries qc = fl(q.c) instead of qn and dq (QN = (qc, ||q|| up, pair,
// qc)), and the filter is Cauchy-Schwarz: -q.x >= -q.c - ||q|| ||x - c|| -
// slack, slack = 1.01 u |qc| + (d + 2) u ||q|| rmx[p] (search.cpp's own rounding
// of the exact sum, rmx the list's max ||x||), so a list whose largest radius
// lies below (-qc - slack - T) / ||q|| holds no candidate with exact score <= T.
// G: lanes per pair (16; 64 for long rows, k_pairs at d > 256 -- the dims loop is
// then a quarter as long: GIST1M's 960 dims were 60 dependent-load steps per lane)
// pair_record in two halves, so a kernel can run the record's sums (which do not
// depend on the seed bound) while other waves compute that bound (k_seed_w):
// pair_sums -- the double sums of the pair's 16 (G) lanes and the QH row, every lane
// holds the pair's totals; pair_finish -- the filter under qb and the record writes.
struct PairSums {
    double s, t, e;
    float2 ts;  // (estimate) this lane's sample tile of the list
    int lsz;    // (estimate) the list's size
};
template <int G = 16>
__device__ __forceinline__ PairSums pair_sums(const float *Q, int64_t d, int64_t pair, bool valid, int praw,
                                              int n_lists, const float *pivot, int centred, const float2 *lstat,
                                              const float4 *QN, float *QE, uint16_t *QH, int64_t dpad,
                                              const int32_t *est_size = nullptr, const float2 *est_samp = nullptr) {
    const bool ipm = centred == 2;
    const int sub = threadIdx.x & (G - 1);
    const int p = praw < n_lists ? praw : -1;  // (an id >= n_lists passes through: k_count reports it)
    (void)valid;  // (Q is the pair's query row)
    PairSums r;
    // (estimate) this lane's sample tile of the list and the list's size, loaded ahead
    const bool est_on = est_size && p >= 0;
    r.ts = est_on && sub < 16 ? est_samp[p * 16 + sub] : make_float2(0.0f, 0.0f);
    r.lsz = est_on ? est_size[p] : 0;
    double s = 0.0, t = 0.0, e = 0.0;
    if (p >= 0 && (QN || lstat)) {
        const float *qr = Q, *pv = pivot ? pivot + (int64_t)p * d : nullptr;
        uint16_t *qh = QH ? QH + pair * dpad : nullptr;
        // (unrolled: 8 iterations' loads in flight together -- a dependent load per
        // iteration made the fused seed + pairs kernel latency-bound)
#pragma unroll 8
        for (int64_t j = sub; j < d; j += G) {
            const float x = qr[j], cv = pv ? pv[j] : 0.0f;
            const float sv = centred == 1 && pv ? x - cv : x;
            if (qh) qh[j] = (uint16_t)bf16_rne_sat(sv);
            const double xc = (double)sv;
            s = __builtin_fma(xc, xc, s);
            if (QE) {
                const double rr = (double)(sv - __uint_as_float(bf16_rne_sat(sv) << 16));
                e = __builtin_fma(rr, rr, e);
            }
            if (pv) {
                if (ipm) {  // q.c
                    t = __builtin_fma((double)x, (double)cv, t);
                } else {
                    const double df = (double)x - (double)cv;
                    t = __builtin_fma(df, df, t);
                }
            }
        }
        if (qh)
            for (int64_t j = d + sub; j < dpad; j += G) qh[j] = 0;
    }
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {  // within the pair's lanes
        s += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, s), m));
        t += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, t), m));
        e += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, e), m));
    }
    r.s = s;
    r.t = t;
    r.e = e;
    return r;
}

template <int G = 16>
__device__ __forceinline__ int pair_finish(const PairSums &r, int64_t d, int64_t pair, bool valid, int praw,
                                           int nprobe, int n_lists, int centred, const float2 *lstat, uint32_t qb,
                                           int32_t *probe_live, float4 *QN, float *QE, float *pqn,
                                           const int32_t *est_size = nullptr, const float *rmx = nullptr) {
    const bool ipm = centred == 2;
    const int sub = threadIdx.x & (G - 1);
    const int p = praw < n_lists ? praw : -1;
    const bool est_on = est_size && p >= 0;
    const double s = r.s, t = r.t, e = r.e;
    // (the interval math runs in lane 0 of the pair only, unless the estimate needs it in all 16)
    if (!est_size && (sub != 0 || !valid)) return 0;
    int live = p;
    const float dq = ipm ? (float)t : (float)__builtin_sqrt(t);  // (IP: qc = fl(q.c))
    const double qnd = __builtin_sqrt(s);
    float fa = -__builtin_inff(), fb = __builtin_inff();  // the triangle (IP: Cauchy-Schwarz) interval
    if (ipm && p >= 0 && lstat && rmx && (int)(pair % nprobe) >= 1 && qb != ~0u && qnd > 0.0) {
        const double dd = (double)d, T = (double)ord2f(qb);
        if (T < 1e300) {
            const double qnu = qnd * (1.0 + 0x1p-40);
            const double slack = (1.01 * __builtin_fabs(t) + (dd + 2.0) * qnu * (double)rmx[p]) * kU * 1.01 + 0x1p-120;
            double A = (-t - slack - T) / qnu;
            A -= __builtin_fabs(A) * 0x1p-40 + 0x1p-120;
            fa = __double2float_rd(A);
            const float2 ls = lstat[p];
            if (ls.y < fa) live = -1;
        }
    } else if (!ipm && p >= 0 && lstat && (int)(pair % nprobe) >= 1) {
        const double dd = (double)d, F = 1.0 - (dd + 4.0) * kU;
        if (qb != ~0u && F > 0.5) {
            const double T = (double)ord2f(qb);
            if (T < 1e300) {
                const double rad = __builtin_sqrt((fmax(T, 0.0) + dd * 0x1p-140) / F) * (1.0 + 0x1p-40);
                double A = (double)dq * (1.0 - 0x1p-22) - rad, B = (double)dq * (1.0 + 0x1p-22) + rad;
                A -= __builtin_fabs(A) * 0x1p-50;
                B += __builtin_fabs(B) * 0x1p-50;
                fa = __double2float_rd(A);
                fb = __double2float_ru(B);
                const float2 ls = lstat[p];
                if (ls.y < fa || ls.x > fb) live = -1;
            }
        }
    }
    int est = 0;
    if (est_size) {
        const bool hit = est_on && valid && live >= 0 && sub < 16 && !(r.ts.y < fa || r.ts.x > fb);
        const unsigned long long bal = __ballot(hit);
        const int hits = __builtin_popcount((unsigned)((bal >> (threadIdx.x & (64 - G))) & 0xffffu));  // (the pair's first 16 lanes)
        est = (int)(((int64_t)((r.lsz + 255) / 256) * hits) / 16);  // blocks of 4 tiles
    }
    if (sub != 0 || !valid) return est;
    probe_live[pair] = praw >= n_lists ? praw : live;
    if (live < 0) return est;
    const float qnu = __double2float_ru(qnd * (1.0 + 0x1p-40));
    if (QN) QN[pair] = make_float4(ipm ? dq : (float)s, qnu, __int_as_float((int)pair), dq);
    if (QE) QE[pair] = __double2float_ru(__builtin_sqrt(e) * (1.0 + 0x1p-40));
    if (pqn) pqn[pair] = qnu;
    return est;
}

template <int G = 16>
__device__ __forceinline__ int pair_record(const float *Q, int64_t d, int64_t pair, bool valid, int praw,
                                           int nprobe, int n_lists, const float *pivot, int centred,
                                           const float2 *lstat, uint32_t qb, int32_t *probe_live, float4 *QN,
                                           float *QE, float *pqn, uint16_t *QH, int64_t dpad,
                                           const int32_t *est_size = nullptr, const float2 *est_samp = nullptr,
                                           const float *rmx = nullptr) {
    const int64_t q = valid ? pair / nprobe : 0;
    const PairSums r = pair_sums<G>(Q + q * d, d, pair, valid, praw, n_lists, pivot, centred, lstat, QN, QE, QH,
                                    dpad, est_size, est_samp);
    return pair_finish<G>(r, d, pair, valid, praw, nprobe, n_lists, centred, lstat, qb, probe_live, QN, QE, pqn,
                          est_size, rmx);
}

}  // namespace lira
