// lira_rank.hip -- query -> centroid ranking and probe selection (gfx950).
//
//   k_centroid_dist   exact search.cpp distances: sqrt of the sequential fp32
//                     sum of fl(q-c)^2 (search.cpp:220-235), optional
//                     standardisation (search.cpp:238-250).  Feeds the probing
//                     MLP and the threshold probe (search.cpp:430-466).
//   k_centroid_gemm   MFMA (v_mfma_f32_32x32x2_f32) ||q||^2+||c||^2-2q.c with a
//                     per-query error bound; the batched ranking GEMM.
//   k_rank_select     nearest-nprobe from the GEMM, exact boundary re-check so
//                     the result equals ranking by the exact distances.
//   k_select_probes   nearest / threshold(>=, argmax fallback) / threshold(>)
//                     over a score matrix (search.cpp:447-466, LIRA_smallscale.py:206).
#include <algorithm>
#include <string>

#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

// fp32 sqrt, correctly rounded: LLVM's lowering of the IEEE sqrt written out
// (v_sqrt_f32 is within 1 ulp; the two fma residuals pick the nearest of s and
// its neighbours; values below 2^-96 are scaled by 2^32 first).  hipcc lowered
// __fsqrt_rn to the bare 1-ulp form in k_rank_exact_dc (not in the others), and a
// (sqrt, index) key 1 ulp off changes which of two near-equal centroids ranks
// first; every distance and key in this file uses this one.
__device__ __forceinline__ float sqrt_rn_f32(float x) {
    const bool scale = x < 0x1p-96f;
    const float xs = scale ? x * 0x1p+32f : x;
    const float s = __builtin_amdgcn_sqrtf(xs);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, xs), rp = __builtin_fmaf(-sp, s, xs);
    float r = rp > 0.0f ? sp : rm <= 0.0f ? sm : s;
    r = scale ? r * 0x1p-16f : r;
    return (xs == 0.0f || !(xs < __builtin_inff())) ? xs : r;  // (+-0, +inf, NaN as they are)
}


// ---------------------------------------------------------------- exact dist
// Tiled like a GEMM: a workgroup owns 64 queries x 64 centroids, stages 32-dim
// slabs of both (coalesced row loads, transposed into LDS), and each thread
// keeps 4 x 4 pairs' sums -- every one search.cpp's own sequential fp32 sum of
// fl(q_j - c_j)^2 in j order (no contraction: -ffp-contract=off), then sqrt
// and the optional standardisation.
__global__ __launch_bounds__(256) void k_centroid_dist(const float *__restrict__ q, int64_t nq,
                                                       const float *__restrict__ cent, int nb,
                                                       int64_t d, const float *mean,
                                                       const float *scale, float *out) {
    __shared__ __attribute__((aligned(16))) float Qs[32][68], Cs[32][68];  // [dim][row], padded
    const int tid = threadIdx.x;
    const int64_t q0 = (int64_t)blockIdx.x * 64;
    const int c0 = blockIdx.y * 64;
    const int tq = (tid & 15) * 4, tc = (tid >> 4) * 4;
    float acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = 0.0f;
    for (int64_t j0 = 0; j0 < d; j0 += 32) {
        const int nj = (int)min<int64_t>(32, d - j0);
        for (int i = tid; i < 64 * 32; i += 256) {
            const int r = i >> 5, jj = i & 31;
            Qs[jj][r] = q0 + r < nq && jj < nj ? q[(q0 + r) * d + j0 + jj] : 0.0f;
            Cs[jj][r] = c0 + r < nb && jj < nj ? cent[(int64_t)(c0 + r) * d + j0 + jj] : 0.0f;
        }
        __syncthreads();
        for (int jj = 0; jj < nj; ++jj) {
            const float4 qa = *(const float4 *)&Qs[jj][tq];
            const float4 ca = *(const float4 *)&Cs[jj][tc];
            const float qv[4] = {qa.x, qa.y, qa.z, qa.w}, cv[4] = {ca.x, ca.y, ca.z, ca.w};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const float df = qv[a] - cv[b];
                    acc[a][b] = acc[a][b] + df * df;
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int64_t qi = q0 + tq + a;
        if (qi >= nq) continue;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int cb = c0 + tc + b;
            if (cb >= nb) continue;
            float r = sqrt_rn_f32(acc[a][b]);
            if (mean) {
                float s = scale[cb];
                if (s == 0.0f) s = 1.0f;
                r = __fdiv_rn(r - mean[cb], s);
            }
            out[qi * nb + cb] = r;
        }
    }
}

// ---------------------------------------------------------------- MFMA GEMM
// Workgroup = 4 waves = 64 queries x 64 centroids; wave (wr, wc) owns a 32x32
// accumulator of v_mfma_f32_32x32x2_f32 (A: lane -> row lane&31, k lane>>5;
// B: k lane>>5, col lane&31; C: col lane&31, row (r&3)+8(r>>2)+4(lane>>5)).
// Operands go through LDS in 64-dim chunks, loaded as coalesced float4 (16
// lanes per 256-B row segment; VEC = d % 4 == 0, else scalar loads).  The
// squared norms are accumulated in registers from the same loads (each thread
// owns 4 query rows and 4 centroid rows x 4 dims of a chunk) and reduced over
// the 16 lanes of a row at the end -- no serial pass over LDS.
typedef float f32x16 __attribute__((ext_vector_type(16)));
static constexpr int kGK = 64;        // dims per LDS chunk
static constexpr int kGLd = kGK + 2;  // padded row: the MFMA reads (32 rows x 2 dims) hit 64 banks

template <bool VEC>
__global__ __launch_bounds__(256) void k_centroid_gemm(const float *__restrict__ q, int64_t nq,
                                                       const float *__restrict__ cent, int nb,
                                                       int64_t d, float *out_sq, float *out_err) {
    __shared__ __attribute__((aligned(16))) float Qs[64 * kGLd];
    __shared__ __attribute__((aligned(16))) float Cs[64 * kGLd];  // 8-B aligned rows
    __shared__ float nrm[128];  // [0,64) query norms, [64,128) centroid norms
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int64_t q0 = (int64_t)blockIdx.x * 64;
    const int c0 = blockIdx.y * 64;
    const int lr = tid >> 4, l4 = (tid & 15) * 4;  // load role: rows lr + 16 i, dims l4..l4+3
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    float nq_acc[4] = {0.f, 0.f, 0.f, 0.f}, nc_acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t k0 = 0; k0 < d; k0 += kGK) {
        float4 vq[4], vc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = lr + 16 * i;
            const int64_t qr = q0 + r, kk = k0 + l4;
            const int cr = c0 + r;
            if (VEC) {
                vq[i] = qr < nq && kk < d ? *(const float4 *)(q + qr * d + kk) : make_float4(0.f, 0.f, 0.f, 0.f);
                vc[i] = cr < nb && kk < d ? *(const float4 *)(cent + (int64_t)cr * d + kk)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float t[4], u[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    t[e] = qr < nq && kk + e < d ? q[qr * d + kk + e] : 0.f;
                    u[e] = cr < nb && kk + e < d ? cent[(int64_t)cr * d + kk + e] : 0.f;
                }
                vq[i] = make_float4(t[0], t[1], t[2], t[3]);
                vc[i] = make_float4(u[0], u[1], u[2], u[3]);
            }
        }
        __syncthreads();  // the previous chunk's MFMA reads are done
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = lr + 16 * i;
            *(float2 *)&Qs[r * kGLd + l4] = make_float2(vq[i].x, vq[i].y);
            *(float2 *)&Qs[r * kGLd + l4 + 2] = make_float2(vq[i].z, vq[i].w);
            *(float2 *)&Cs[r * kGLd + l4] = make_float2(vc[i].x, vc[i].y);
            *(float2 *)&Cs[r * kGLd + l4 + 2] = make_float2(vc[i].z, vc[i].w);
            nq_acc[i] = fmaf(vq[i].x, vq[i].x, fmaf(vq[i].y, vq[i].y, fmaf(vq[i].z, vq[i].z, fmaf(vq[i].w, vq[i].w, nq_acc[i]))));
            nc_acc[i] = fmaf(vc[i].x, vc[i].x, fmaf(vc[i].y, vc[i].y, fmaf(vc[i].z, vc[i].z, fmaf(vc[i].w, vc[i].w, nc_acc[i]))));
        }
        __syncthreads();
        const float *qa = Qs + (wr * 32 + (lane & 31)) * kGLd + (lane >> 5);
        const float *cb_ = Cs + (wc * 32 + (lane & 31)) * kGLd + (lane >> 5);
#pragma unroll
        for (int kk = 0; kk < kGK; kk += 2)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(qa[kk], cb_[kk], acc, 0, 0, 0);
    }
    // row norms: reduce over the 16 lanes that loaded a row
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            nq_acc[i] += __shfl_xor(nq_acc[i], o);
            nc_acc[i] += __shfl_xor(nc_acc[i], o);
        }
    }
    if ((tid & 15) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            nrm[lr + 16 * i] = nq_acc[i];
            nrm[64 + lr + 16 * i] = nc_acc[i];
        }
    }
    __syncthreads();
    // |A - R| <= (2 gamma_d + 4u)(nq + nc) and |E - R| <= 2 gamma_{d+3}(nq + nc)
    // (R real, E = search.cpp's sequential sum; any summation order of the
    // norms and the dot stays within gamma_d), so |A - E| <= (4d + 10)u(nq + nc);
    // 8(d+8)u leaves room for sqrt() merging nearby E values into one float.
    const float ebound = 8.0f * (float)(d + 8) * 5.9604645e-08f;
    const int col = lane & 31;
    const int cb = c0 + wc * 32 + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        int64_t qr = q0 + wr * 32 + row;
        float nq_ = nrm[wr * 32 + row], nc_ = nrm[64 + wc * 32 + col];
        float v = (nq_ + nc_) - 2.0f * acc[r];
        if (qr < nq && cb < nb) out_sq[qr * nb + cb] = v;
    }
    // the bound grows with ||c||^2: per query row, with the block's largest
    // in-range centroid norm; one column block (nb <= 64) stores it, several
    // take the max over blocks (the caller zeroed out_err)
    if (out_err && w == 0) {
        float mx = c0 + lane < nb ? nrm[64 + lane] : 0.0f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        const int64_t qr = q0 + lane;
        if (qr < nq) {
            const float e = ebound * (nrm[lane] + mx) + 1e-30f;
            if (gridDim.y == 1) out_err[qr] = e;
            else atomicMax((unsigned int *)&out_err[qr], __float_as_uint(e));
        }
    }
}

// search.cpp:220-235's sequential sum of fl(q_j - c_j)^2 over one centroid row, 16
// dims of loads per step where both rows are 16-B aligned
__device__ __forceinline__ float exact_l2_row(const float *qr, const float *cr, int64_t d) {
    float acc = 0.0f;
    int64_t j = 0;
    if ((((uintptr_t)cr | (uintptr_t)qr) & 15) == 0) {
        // qr is wave-uniform (k_rank_select's query row): constant-address-space reads,
        // so its pieces come by scalar loads and the VGPRs hold the centroid pieces only
        typedef float f4v __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(4))) f4v cf4;
        cf4 *q4 = (cf4 *)qr;
#pragma unroll 2
        for (; j + 16 <= d; j += 16) {
            float4 cv[4];
            f4v qv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                cv[e] = *(const float4 *)(cr + j + 4 * e);
                qv[e] = q4[(j >> 2) + e];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float df = qv[e].x - cv[e].x;
                acc = acc + df * df;
                df = qv[e].y - cv[e].y;
                acc = acc + df * df;
                df = qv[e].z - cv[e].z;
                acc = acc + df * df;
                df = qv[e].w - cv[e].w;
                acc = acc + df * df;
            }
        }
    }
    for (; j < d; ++j) {
        const float df = qr[j] - cr[j];
        acc = acc + df * df;
    }
    return acc;
}

// -------------------------------------------------------- nearest, re-checked
// One wave per query.  1) T = nprobe-th smallest approximate value; 2) every b
// with A_b <= T + 2M (M = the query's error bound) gets its exact search.cpp
// distance; 3) exact (sqrt(l2), b) top-nprobe.  Any b of the exact top-nprobe
// satisfies A_b <= T + 2M, so the result equals ranking all B exactly.
template <int R>
__global__ __launch_bounds__(256) void k_rank_select(const float *__restrict__ A,
                                                     const float *__restrict__ err,
                                                     const float *__restrict__ q, int64_t nq,
                                                     const float *__restrict__ cent, int nb,
                                                     int64_t d, int nprobe, int32_t *out) {
    __shared__ uint32_t s_cand[4][64];
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (qi >= nq) return;
    const float *arow = A + qi * nb;
    // T: any value with at least min(nprobe, nb) approximate values <= T works (the
    // candidates are every b with A_b <= T + 2M, re-checked exactly; T >= the nprobe-th
    // smallest keeps every member of the exact top-nprobe among them).  nb <= 1024: the
    // row in registers (16 per lane, one round of loads) and T by bisection on the
    // value range, stopped once few extra values pass -- the nprobe-th key by u64 bitonic
    // merges of the 16 batches was ~3.7 k VALU instructions per query (BIGANN-100M,
    // B = 1024: VALU-bound at ~60 us per 10 k queries).  Larger nb: those merges.
    constexpr int NV = 16;
    float lim;
    if (nb <= 64 * NV) {
        float av[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int b = 64 * i + lane;
            av[i] = b < nb ? arow[b] : __builtin_nanf("");
        }
        float lo = __builtin_inff(), hi = -__builtin_inff();
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            if (av[i] == av[i]) {
                lo = fminf(lo, av[i]);
                hi = fmaxf(hi, av[i]);
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            lo = fminf(lo, __shfl_xor(lo, m, 64));
            hi = fmaxf(hi, __shfl_xor(hi, m, 64));
        }
        auto count_le = [&](float t) __attribute__((always_inline)) {
            int c = 0;
#pragma unroll
            for (int i = 0; i < NV; ++i) c += av[i] <= t;  // (NaN: never)
            return (int)wave_sum_u64((u64)c);
        };
        const int target = min(nprobe, nb);
        // invariant: count(<= hi) >= target; a pass keeps the lower half while it holds
        for (int it = 0; it < 24 && hi > lo; ++it) {
            const float mid = lo + (hi - lo) * 0.5f;
            if (!(mid > lo && mid < hi)) break;
            const int c = count_le(mid);
            if (c >= target) hi = mid; else lo = mid;
            if (c >= target && c <= target + 16) break;  // (few extra candidates: good enough)
        }
        lim = hi < __builtin_inff() ? hi + 2.0f * err[qi] * 1.0001f : __builtin_inff();
    } else {
        u64 lst[R];
#pragma unroll
        for (int r = 0; r < R; ++r) lst[r] = kEmptyKey;
        for (int b0 = 0; b0 < nb; b0 += 64) {
            const int b = b0 + lane;
            const u64 key = b < nb ? make_key(arow[b], b) : kEmptyKey;
            const u64 thr = wave_list_at<R>(lst, nprobe - 1);
            if (__ballot(key < thr)) wave_merge_batch<R>(lst, key);
        }
        const u64 tk = wave_list_at<R>(lst, nprobe - 1);
        lim = tk == kEmptyKey ? __builtin_inff() : key_score(tk) + 2.0f * err[qi] * 1.0001f;
    }
    const float *qr = q + qi * d;
    u64 fin[R];
#pragma unroll
    for (int r = 0; r < R; ++r) fin[r] = kEmptyKey;
    // the candidates (A_b <= lim: ~nprobe of them) compacted into the wave's LDS list
    // first, then re-checked 64 at a time, one per lane: walking the B / 64 batches
    // with a re-check each (a couple of live lanes per batch at B = 1024) made every
    // query a chain of 16 dependent d-long sums (BIGANN-100M: 0.32 ms per 10 k queries)
    uint32_t *cl = s_cand[threadIdx.x >> 6];
    int nc = 0;
    auto flush = [&]() __attribute__((always_inline)) {
        u64 key = kEmptyKey;
        if (lane < nc) {
            const int b = (int)cl[lane];
            key = make_key(sqrt_rn_f32(exact_l2_row(qr, cent + (int64_t)b * d, d)), b);
        }
        wave_merge_batch<R>(fin, key);
        nc = 0;
        __builtin_amdgcn_wave_barrier();
    };
    for (int c0 = 0; c0 < nb; c0 += 64 * NV) {
        float av[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int b = c0 + 64 * i + lane;
            av[i] = b < nb ? arow[b] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int b = c0 + 64 * i + lane;
            if (c0 + 64 * i >= nb) break;
            const bool cand = b < nb && av[i] <= lim;
            const u64 m = __ballot(cand);
            const int n = popc64(m);
            if (!n) continue;
            if (nc + n > 64) flush();
            if (cand) cl[nc + mbcnt64(m)] = (uint32_t)b;
            nc += n;
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (nc) flush();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int e = r * 64 + lane;
        if (e < nprobe) out[qi * nprobe + e] = fin[r] == kEmptyKey ? -1 : key_gid(fin[r]);
    }
}

// nb <= 64 (one centroid per lane): the threshold from a 32-bit sort of the
// approximate values (no index tie-break is needed for a value), and the exact
// top-nprobe by counting ranks over the few re-checked lanes (the u64 bitonic
// sorts of k_rank_select were most of its time: SIFT1M 26 us per 10 k queries)
__global__ __launch_bounds__(256) void k_rank_select64(const float *__restrict__ A, const float *__restrict__ err,
                                                       const float *__restrict__ q, int64_t nq,
                                                       const float *__restrict__ cent, int nb, int64_t d,
                                                       int nprobe, int32_t *out) {
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq) return;
    const bool ok = lane < nb;
    const float av = ok ? A[qi * nb + lane] : __builtin_inff();
    const uint32_t sorted = wave_sort64_u32(ok ? f2ord(av) : ~0u);
    const uint32_t tk = (uint32_t)__shfl((int)sorted, min(nprobe, nb) - 1, 64);
    const float lim = ord2f(tk) + 2.0f * err[qi] * 1.0001f;
    const bool cand = ok && av <= lim;
    u64 key = kEmptyKey;
    if (cand) {  // search.cpp:220-235's sequential sum
        const float *qr = q + qi * d, *cr = cent + (int64_t)lane * d;
        float acc = 0.0f;
        int64_t j = 0;
        if ((((uintptr_t)cr | (uintptr_t)qr) & 15) == 0) {
            for (; j + 16 <= d; j += 16) {
                float4 cv[4], qv[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    cv[e] = *(const float4 *)(cr + j + 4 * e);
                    qv[e] = *(const float4 *)(qr + j + 4 * e);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float df = qv[e].x - cv[e].x;
                    acc = acc + df * df;
                    df = qv[e].y - cv[e].y;
                    acc = acc + df * df;
                    df = qv[e].z - cv[e].z;
                    acc = acc + df * df;
                    df = qv[e].w - cv[e].w;
                    acc = acc + df * df;
                }
            }
        }
        for (; j < d; ++j) {
            const float df = qr[j] - cr[j];
            acc = acc + df * df;
        }
        key = make_key(sqrt_rn_f32(acc), lane);
    }
    // rank of my key among the candidates' (keys are distinct: the index breaks ties)
    u64 cm = __ballot(cand);
    const int ncand = __popcll(cm);
    int rank = 0;
    while (cm) {
        const int j = __builtin_ctzll(cm);
        cm &= cm - 1;
        const u64 kj = ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), j) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, j);
        rank += kj < key;
    }
    int32_t *o = out + qi * nprobe;
    if (cand && rank < nprobe) o[rank] = lane;
    for (int e = ncand + lane; e < nprobe; e += 64) o[e] = -1;
}

// nb <= 64, d % 4 == 0, d <= 256: the ranking in ONE exact pass, no GEMM and no
// re-check -- lane b = centroid b, whose rows sit transposed in LDS as float4
// [d/4][64] (lane b reads dims 4j..4j+3 of its own centroid, conflict-free);
// the query row comes in by scalar loads (wave-uniform).  Every distance is
// search.cpp:220-235's sequential fp32 sum of fl(q_j - c_j)^2 in j order, so
// the (sqrt, index) keys are the ones k_rank_select64 re-checks, and one u64
// sort of the wave's 64 keys gives the nearest nprobe.  64 distances x d dims
// is less VALU work than the GEMM's launch plus the re-check's (SIFT1M, 10 k
// queries: k_centroid_gemm 8 us + k_rank_select64 23 us before).
// 8 waves per workgroup (the 32 KB LDS image staged once per 8 or 16 queries);
// qpw queries per wave, one after the other (1 for small batches: the chain of a
// wave's queries, not the VALU work, set the time -- 8 per wave ran 31 us at 10 k
// queries and 28 us at 1.25 k)
__global__ __launch_bounds__(512) void k_rank_exact64(const float *__restrict__ q, int64_t nq,
                                                      const float *__restrict__ cent, int nb, int64_t d,
                                                      int nprobe, int qpw, int32_t *out) {
    extern __shared__ float4 Cs[];  // [d/4][64], then the workgroup's 8 qpw query rows [8 qpw][d/4]
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nd4 = (int)(d >> 2);
    float4 *Qs = Cs + 64 * nd4;
    const int64_t qb0 = (int64_t)blockIdx.x * (8 * qpw);
    // coalesced row reads (consecutive threads: consecutive float4 of one row); the
    // workgroup's query rows come in the same round, so a wave's chain per query is
    // LDS reads only (its rows by wave-uniform global loads, four rounds of eight 16-B
    // loads per query, were most of the kernel's time: SIFT1M 22 us per 10 k queries)
    for (int i = tid; i < 64 * nd4; i += 512) {
        const int b = i / nd4, j4 = i - b * nd4;
        Cs[j4 * 64 + b] = b < nb ? *(const float4 *)(cent + (int64_t)b * d + 4 * j4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int i = tid; i < 8 * qpw * nd4; i += 512) {
        const int64_t qi = qb0 + i / nd4;
        Qs[i] = qi < nq ? *(const float4 *)(q + qi * d + 4 * (i % nd4)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const int64_t q0 = qb0 + w * qpw;
    for (int r = 0; r < qpw; ++r) {
        const int64_t qi = q0 + r;
        if (qi >= nq) break;
        const float4 *qr = Qs + (int64_t)(w * qpw + r) * nd4;
        float acc = 0.0f;
#pragma unroll 8
        for (int j4 = 0; j4 < nd4; ++j4) {
            const float4 qv = qr[j4], cv = Cs[j4 * 64 + lane];
            float df = qv.x - cv.x;
            acc = acc + df * df;
            df = qv.y - cv.y;
            acc = acc + df * df;
            df = qv.z - cv.z;
            acc = acc + df * df;
            df = qv.w - cv.w;
            acc = acc + df * df;
        }
        const u64 key = wave_sort64(lane < nb ? make_key(sqrt_rn_f32(acc), lane) : kEmptyKey);
        int32_t *o = out + qi * nprobe;
        if (lane < nprobe) o[lane] = key == kEmptyKey ? -1 : key_gid(key);
        for (int e = 64 + lane; e < nprobe; e += 64) o[e] = -1;
    }
}
static bool rank_exact64_ok(const float *q, const float *cent, int64_t nb, int64_t d) {
    return nb <= 64 && d % 4 == 0 && d <= 256 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)cent & 15) == 0;
}

// The same one-pass exact ranking for 64 < nb <= 256 or d > 256 (GIST1M: B =
// 128, d = 960; DEEP10M: B = 256): CPL centroids per lane (lane b holds
// centroids b, b + 64, ..), the centroid rows staged transposed through LDS in
// chunks of DC4 float4 columns ([DC4][64 CPL], 64 KB) -- every query of the
// workgroup (one per wave) consumes a chunk before the next is staged, so the
// partial sums carry over and each one stays search.cpp:220-235's sequential
// fp32 sum in dim order.  Then one sort of the wave's 64 CPL (sqrt, index) keys.
// Replaces the MFMA GEMM + boundary re-check there (GIST1M 1 k queries:
// k_centroid_gemm + k_rank_select 68 us).
template <int CPL>
__global__ __launch_bounds__(512) void k_rank_exact_dc(const float *__restrict__ q, int64_t nq,
                                                      const float *__restrict__ cent, int nb, int64_t d,
                                                      int nprobe, int32_t *out) {
    constexpr int NC = 64 * CPL, DC4 = 4096 / NC;  // (64 KB of LDS)
    __shared__ float4 Cs[DC4 * NC];
    const int tid = threadIdx.x, lane = tid & 63, nw = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nd4 = (int)(d >> 2);
    const int64_t qi = (int64_t)blockIdx.x * nw + w;
    const float4 *qr = (const float4 *)(q + (qi < nq ? qi : 0) * d);
    float acc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc[c] = 0.0f;
    for (int j0 = 0; j0 < nd4; j0 += DC4) {
        const int nd = min(DC4, nd4 - j0);
        __syncthreads();  // (the previous chunk is consumed)
        for (int i = tid; i < NC * nd; i += blockDim.x) {  // consecutive threads: consecutive float4 of one row
            const int b = i / nd, jj = i - b * nd;
            Cs[jj * NC + b] = b < nb ? *(const float4 *)(cent + (int64_t)b * d + 4 * (j0 + jj)) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __syncthreads();
        if (qi < nq) {
#pragma unroll 4
            for (int jj = 0; jj < nd; ++jj) {
                const float4 qv = qr[j0 + jj];
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const float4 cv = Cs[jj * NC + c * 64 + lane];
                    float df = qv.x - cv.x;
                    acc[c] = acc[c] + df * df;
                    df = qv.y - cv.y;
                    acc[c] = acc[c] + df * df;
                    df = qv.z - cv.z;
                    acc[c] = acc[c] + df * df;
                    df = qv.w - cv.w;
                    acc[c] = acc[c] + df * df;
                }
            }
        }
    }
    if (qi >= nq) return;
    u64 key[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) key[c] = c * 64 + lane < nb ? make_key(sqrt_rn_f32(acc[c]), c * 64 + lane) : kEmptyKey;
    wave_sort<CPL>(key);  // element r * 64 + lane in key[r]
    int32_t *o = out + qi * nprobe;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
        if (c * 64 + lane < nprobe) o[c * 64 + lane] = key[c] == kEmptyKey ? -1 : key_gid(key[c]);
    for (int e = NC + lane; e < nprobe; e += 64) o[e] = -1;
}
static int rank_exact_dc_cpl(const float *q, const float *cent, int64_t nb, int64_t d) {
    if (d % 4 != 0 || ((uintptr_t)q & 15) != 0 || ((uintptr_t)cent & 15) != 0) return 0;
    return nb <= 64 ? 1 : nb <= 128 ? 2 : nb <= 256 ? 4 : 0;
}

// -------------------------------------------------------------- probe select
template <int R>
__global__ __launch_bounds__(256) void k_select_nearest(const float *__restrict__ s, int64_t n,
                                                        int nb, int np, int32_t *out,
                                                        int32_t *out_np) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const float *row = s + i * nb;
    u64 lst[R];
#pragma unroll
    for (int r = 0; r < R; ++r) lst[r] = kEmptyKey;
    for (int b0 = 0; b0 < nb; b0 += 64) {
        int b = b0 + lane;
        u64 key = b < nb ? make_key(row[b], b) : kEmptyKey;
        u64 thr = wave_list_at<R>(lst, np - 1);
        if (__ballot(key < thr)) wave_merge_batch<R>(lst, key);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int e = r * 64 + lane;
        if (e < np) out[i * np + e] = lst[r] == kEmptyKey ? -1 : key_gid(lst[r]);
    }
    if (out_np && lane == 0) out_np[i] = min(np, nb);
}

// threshold: ascending bucket order; ge = (>=, argmax fallback) else (>, none)
__global__ __launch_bounds__(256) void k_select_threshold(const float *__restrict__ s, int64_t n,
                                                          int nb, float thr, int ge, int maxp,
                                                          int32_t *out, int32_t *out_np) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const float *row = s + i * nb;
    int32_t *o = out + i * maxp;
    int m = 0;
    float best = -__builtin_inff();
    int bestb = 0x7fffffff;
    for (int b0 = 0; b0 < nb; b0 += 64) {
        int b = b0 + lane;
        float v = b < nb ? row[b] : 0.0f;
        bool take = b < nb && (ge ? v >= thr : v > thr);
        u64 bal = __ballot(take);
        int pos = m + mbcnt64(bal);
        if (take && pos < maxp) o[pos] = b;
        m += popc64(bal);
        // running argmax, first max wins (search.cpp:456-466: strict >)
        if (b < nb && (v > best || (v == best && b < bestb))) {
            best = v;
            bestb = b;
        }
    }
    if (ge && m == 0) {
        // wave argmax over (best, bestb): larger value, then smaller bucket
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            float ov = __shfl_xor(best, off, 64);
            int ob = __shfl_xor(bestb, off, 64);
            if (ov > best || (ov == best && ob < bestb)) {
                best = ov;
                bestb = ob;
            }
        }
        // search.cpp seeds with bucket 0 and replaces only on strictly greater
        // values: a NaN in bucket 0 (or a row of NaNs) probes bucket 0
        if (bestb == 0x7fffffff || row[0] != row[0]) bestb = 0;
        if (lane == 0) o[0] = bestb;
        m = 1;
    }
    const int mm = min(m, maxp);
    for (int e = mm + lane; e < maxp; e += 64) o[e] = -1;
    if (out_np && lane == 0) out_np[i] = mm;
}

// The same selection with the probes ordered by descending score (ties ->
// smaller bucket) instead of ascending bucket: the set is identical, and the
// scan -- whose results do not depend on slot order -- then meets each
// query's most probable partition first (its seed bound and its nearest-slot
// group; LIRA_PROBE_BY_SCORE).  Truncation at maxp keeps the highest scores.
template <int R>
__global__ __launch_bounds__(256) void k_select_threshold_sorted(const float *__restrict__ s, int64_t n, int nb,
                                                                 float thr, int ge, int maxp, int32_t *out,
                                                                 int32_t *out_np) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const float *row = s + i * nb;
    int32_t *o = out + i * maxp;
    u64 lst[R];
#pragma unroll
    for (int r = 0; r < R; ++r) lst[r] = kEmptyKey;
    int m = 0;
    float best = -__builtin_inff();
    int bestb = 0x7fffffff;
    for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + lane;
        const float v = b < nb ? row[b] : 0.0f;
        const bool take = b < nb && (ge ? v >= thr : v > thr);
        m += popc64(__ballot(take));
        const u64 key = take ? ((u64)(~f2ord(v)) << 32) | (uint32_t)b : kEmptyKey;
        const u64 tk = wave_list_at<R>(lst, 64 * R - 1);
        if (__ballot(key < tk)) wave_merge_batch<R>(lst, key);
        if (b < nb && (v > best || (v == best && b < bestb))) {
            best = v;
            bestb = b;
        }
    }
    if (ge && m == 0) {  // argmax fallback, as k_select_threshold
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            float ov = __shfl_xor(best, off, 64);
            int ob = __shfl_xor(bestb, off, 64);
            if (ov > best || (ov == best && ob < bestb)) {
                best = ov;
                bestb = ob;
            }
        }
        if (bestb == 0x7fffffff || row[0] != row[0]) bestb = 0;
        for (int e = lane; e < maxp; e += 64) o[e] = e == 0 ? bestb : -1;
        if (out_np && lane == 0) out_np[i] = 1;
        return;
    }
    const int mm = min(m, maxp);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < maxp) o[e] = e < mm ? (int32_t)(uint32_t)lst[r] : -1;
    }
    if (out_np && lane == 0) out_np[i] = mm;
}

// lira_order_probes: one wave per row; keys (f2ord(key[b]) << 32 | b), -1 slots
// as empty keys (sorted last), one wave-wide sort of the row's R*64 keys.  An
// id >= n_centroids is kept (after the valid ones, before the padding), so the
// scan still sees it and reports LIRA_ERANGE: ordering never changes the set.
template <int R>
__global__ __launch_bounds__(256) void k_order_probes(int32_t *probe, int64_t n, int mp, const float *__restrict__ key,
                                                      int nb) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    int32_t *row = probe + i * mp;
    u64 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        const int b = e < mp ? row[e] : -1;
        v[r] = b < 0 ? kEmptyKey : b < nb ? ((u64)f2ord(key[i * nb + b]) << 32) | (uint32_t)b
                                          : (0xffffffffull << 32) | (uint32_t)b;
    }
    wave_sort<R>(v);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = r * 64 + lane;
        if (e < mp) row[e] = v[r] == kEmptyKey ? -1 : (int32_t)(uint32_t)v[r];
    }
}

static int sel_r(int64_t np) { return np <= 64 ? 1 : np <= 128 ? 2 : np <= 256 ? 4 : -1; }

}  // namespace lira

using namespace lira;

extern "C" {

int lira_centroid_dist(const float *q, int64_t nq, const float *centroids, int64_t n_centroids,
                       int64_t d, const float *scaler_mean, const float *scaler_scale, float *out,
                       void *stream) {
    if (nq < 0 || n_centroids <= 0 || d <= 0) return fail(LIRA_EINVAL, "bad shape");
    if (n_centroids > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "too many centroids");
    if ((scaler_mean == nullptr) != (scaler_scale == nullptr))
        return fail(LIRA_EINVAL, "scaler_mean and scaler_scale must both be set or both NULL");
    if (nq == 0) return LIRA_OK;
    if (!q || !centroids || !out) return fail(LIRA_EINVAL, "NULL buffer");
    if ((nq + 63) / 64 > INT32_MAX || (n_centroids + 63) / 64 > 65535)
        return fail(LIRA_EUNSUPPORTED, "too many queries / centroids for one launch");
    hipLaunchKernelGGL(k_centroid_dist, dim3((unsigned)((nq + 63) / 64), (unsigned)((n_centroids + 63) / 64)),
                       dim3(256), 0, (hipStream_t)stream, q, nq, centroids, (int)n_centroids, d, scaler_mean,
                       scaler_scale, out);
    LIRA_HIP_TRY(hipGetLastError());
    return LIRA_OK;
}

int lira_centroid_gemm(const float *q, int64_t nq, const float *centroids, int64_t n_centroids,
                       int64_t d, float *out_sq, float *out_err, void *stream) {
    if (nq < 0 || n_centroids <= 0 || d <= 0) return fail(LIRA_EINVAL, "bad shape");
    if (n_centroids > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "too many centroids");
    if (nq == 0) return LIRA_OK;
    if (!q || !centroids || !out_sq) return fail(LIRA_EINVAL, "NULL buffer");
    hipStream_t st = (hipStream_t)stream;
    if (out_err && n_centroids > 64) LIRA_HIP_TRY(fill32_async(out_err, 0u, nq * 4, st));  // (max over column blocks)
    dim3 grid((unsigned)((nq + 63) / 64), (unsigned)((n_centroids + 63) / 64));
    if (d % 4 == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)centroids & 15) == 0)
        hipLaunchKernelGGL(k_centroid_gemm<true>, grid, dim3(256), 0, st, q, nq, centroids,
                           (int)n_centroids, d, out_sq, out_err);
    else
        hipLaunchKernelGGL(k_centroid_gemm<false>, grid, dim3(256), 0, st, q, nq, centroids,
                           (int)n_centroids, d, out_sq, out_err);
    LIRA_HIP_TRY(hipGetLastError());
    return LIRA_OK;
}

int lira_rank_workspace_size(int64_t nq, int64_t n_centroids, size_t *bytes) {
    if (!bytes || nq < 0 || n_centroids <= 0) return fail(LIRA_EINVAL, "bad arguments");
    *bytes = (size_t)round_up(nq * n_centroids * 4, 256) + (size_t)round_up(nq * 4, 256);
    return LIRA_OK;
}

int lira_rank_nearest(const float *q, int64_t nq, const float *centroids, int64_t n_centroids,
                      int64_t d, int64_t nprobe, int32_t *out_probe, void *workspace,
                      size_t workspace_bytes, void *stream) {
    if (nq < 0 || n_centroids <= 0 || d <= 0) return fail(LIRA_EINVAL, "bad shape");
    int R = sel_r(nprobe);
    if (nprobe <= 0 || R < 0) return fail(LIRA_EUNSUPPORTED, "nprobe must be in [1, 256]");
    if (nq == 0) return LIRA_OK;
    if (!q || !centroids || !out_probe) return fail(LIRA_EINVAL, "NULL buffer");
    if (rank_exact64_ok(q, centroids, n_centroids, d)) {  // (no workspace needed)
        const int qpw = nq >= 8192 ? 2 : 1;
        const unsigned g = (unsigned)((nq + 8 * qpw - 1) / (8 * qpw));
        static std::atomic<uint64_t> attr{0};  // (d = 256, qpw 4: 64 + 32 KB)
        LIRA_HIP_TRY(set_smem_attr_once(attr, (const void *)k_rank_exact64, 128 * 1024));
        hipLaunchKernelGGL(k_rank_exact64, dim3(g), dim3(512), (size_t)d * 64 * 4 + (size_t)8 * qpw * d * 4,
                           (hipStream_t)stream, q, nq,
                           centroids, (int)n_centroids, d, (int)nprobe, qpw, out_probe);
        LIRA_HIP_TRY(hipGetLastError());
        return LIRA_OK;
    }
    if (const int cpl = rank_exact_dc_cpl(q, centroids, n_centroids, d)) {  // (no workspace needed)
        const int nw = nq >= 4096 ? 8 : 4;  // queries (waves) per workgroup: fewer for small batches
        const unsigned g = (unsigned)((nq + nw - 1) / nw);
        hipStream_t st = (hipStream_t)stream;
        if (cpl == 1)
            hipLaunchKernelGGL(k_rank_exact_dc<1>, dim3(g), dim3(64 * nw), 0, st, q, nq, centroids, (int)n_centroids, d,
                               (int)nprobe, out_probe);
        else if (cpl == 2)
            hipLaunchKernelGGL(k_rank_exact_dc<2>, dim3(g), dim3(64 * nw), 0, st, q, nq, centroids, (int)n_centroids, d,
                               (int)nprobe, out_probe);
        else
            hipLaunchKernelGGL(k_rank_exact_dc<4>, dim3(g), dim3(64 * nw), 0, st, q, nq, centroids, (int)n_centroids, d,
                               (int)nprobe, out_probe);
        LIRA_HIP_TRY(hipGetLastError());
        return LIRA_OK;
    }
    size_t need = 0;
    lira_rank_workspace_size(nq, n_centroids, &need);
    hipStream_t st = (hipStream_t)stream;
    void *ws = workspace;
    bool own = false;
    if (!ws) {
        LIRA_HIP_TRY(hipMallocAsync(&ws, need, st));
        own = true;
    } else if (workspace_bytes < need) {
        return fail(LIRA_EINVAL, "rank workspace too small: need " + std::to_string(need));
    }
    float *A = (float *)ws;
    float *err = (float *)((char *)ws + round_up(nq * n_centroids * 4, 256));
    int rc = lira_centroid_gemm(q, nq, centroids, n_centroids, d, A, err, stream);
    if (rc == LIRA_OK) {
        dim3 g((unsigned)((nq + 3) / 4));
        if (n_centroids <= 64)
            hipLaunchKernelGGL(k_rank_select64, g, dim3(256), 0, st, A, err, q, nq, centroids, (int)n_centroids, d,
                               (int)nprobe, out_probe);
        else if (R == 1)
            hipLaunchKernelGGL(k_rank_select<1>, g, dim3(256), 0, st, A, err, q, nq, centroids,
                               (int)n_centroids, d, (int)nprobe, out_probe);
        else if (R == 2)
            hipLaunchKernelGGL(k_rank_select<2>, g, dim3(256), 0, st, A, err, q, nq, centroids,
                               (int)n_centroids, d, (int)nprobe, out_probe);
        else
            hipLaunchKernelGGL(k_rank_select<4>, g, dim3(256), 0, st, A, err, q, nq, centroids,
                               (int)n_centroids, d, (int)nprobe, out_probe);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = fail(LIRA_EHIP, std::string("k_rank_select: ") + hipGetErrorString(e));
    }
    if (own) hipFreeAsync(ws, st);
    return rc;
}

int lira_order_probes(int32_t *probe, int64_t n, int64_t max_probe, const float *key, int64_t n_centroids,
                      void *stream) {
    if (n < 0 || n_centroids <= 0 || max_probe <= 0) return fail(LIRA_EINVAL, "bad shape");
    const int R = sel_r(max_probe);
    if (R < 0) return fail(LIRA_EUNSUPPORTED, "lira_order_probes supports max_probe <= 256");
    if (n_centroids > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "too many centroids");
    if (n == 0) return LIRA_OK;
    if (!probe || !key) return fail(LIRA_EINVAL, "NULL buffer");
    const dim3 g((unsigned)((n + 3) / 4));
    hipStream_t st = (hipStream_t)stream;
    if (R == 1)
        hipLaunchKernelGGL(k_order_probes<1>, g, dim3(256), 0, st, probe, n, (int)max_probe, key, (int)n_centroids);
    else if (R == 2)
        hipLaunchKernelGGL(k_order_probes<2>, g, dim3(256), 0, st, probe, n, (int)max_probe, key, (int)n_centroids);
    else
        hipLaunchKernelGGL(k_order_probes<4>, g, dim3(256), 0, st, probe, n, (int)max_probe, key, (int)n_centroids);
    LIRA_HIP_TRY(hipGetLastError());
    return LIRA_OK;
}

int lira_select_probes(const float *scores, int64_t n, int64_t n_centroids, int mode, float thr,
                       int64_t max_probe, int32_t *out_probe, int32_t *out_nprobe, void *stream) {
    if (n < 0 || n_centroids <= 0 || max_probe <= 0) return fail(LIRA_EINVAL, "bad shape");
    if (n_centroids > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "too many centroids");
    if (n == 0) return LIRA_OK;
    if (!scores || !out_probe) return fail(LIRA_EINVAL, "NULL buffer");
    hipStream_t st = (hipStream_t)stream;
    dim3 g((unsigned)((n + 3) / 4));
    const bool by_score = (mode & LIRA_PROBE_BY_SCORE) != 0;
    mode &= ~LIRA_PROBE_BY_SCORE;
    if (by_score && (mode == LIRA_PROBE_THRESHOLD_GE || mode == LIRA_PROBE_THRESHOLD_GT)) {
        const int R = sel_r(max_probe);
        if (R < 0) return fail(LIRA_EUNSUPPORTED, "LIRA_PROBE_BY_SCORE supports max_probe <= 256");
        const int ge = mode == LIRA_PROBE_THRESHOLD_GE ? 1 : 0;
        if (R == 1)
            hipLaunchKernelGGL(k_select_threshold_sorted<1>, g, dim3(256), 0, st, scores, n, (int)n_centroids, thr,
                               ge, (int)max_probe, out_probe, out_nprobe);
        else if (R == 2)
            hipLaunchKernelGGL(k_select_threshold_sorted<2>, g, dim3(256), 0, st, scores, n, (int)n_centroids, thr,
                               ge, (int)max_probe, out_probe, out_nprobe);
        else
            hipLaunchKernelGGL(k_select_threshold_sorted<4>, g, dim3(256), 0, st, scores, n, (int)n_centroids, thr,
                               ge, (int)max_probe, out_probe, out_nprobe);
        LIRA_HIP_TRY(hipGetLastError());
        return LIRA_OK;
    }
    if (mode == LIRA_PROBE_NEAREST) {
        int R = sel_r(max_probe);
        if (R < 0) return fail(LIRA_EUNSUPPORTED, "nearest mode supports max_probe <= 256");
        if (R == 1)
            hipLaunchKernelGGL(k_select_nearest<1>, g, dim3(256), 0, st, scores, n, (int)n_centroids,
                               (int)max_probe, out_probe, out_nprobe);
        else if (R == 2)
            hipLaunchKernelGGL(k_select_nearest<2>, g, dim3(256), 0, st, scores, n, (int)n_centroids,
                               (int)max_probe, out_probe, out_nprobe);
        else
            hipLaunchKernelGGL(k_select_nearest<4>, g, dim3(256), 0, st, scores, n, (int)n_centroids,
                               (int)max_probe, out_probe, out_nprobe);
    } else if (mode == LIRA_PROBE_THRESHOLD_GE || mode == LIRA_PROBE_THRESHOLD_GT) {
        if (max_probe > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "max_probe too large");
        hipLaunchKernelGGL(k_select_threshold, g, dim3(256), 0, st, scores, n, (int)n_centroids, thr,
                           mode == LIRA_PROBE_THRESHOLD_GE ? 1 : 0, (int)max_probe, out_probe,
                           out_nprobe);
    } else {
        return fail(LIRA_EINVAL, "unknown probe mode");
    }
    LIRA_HIP_TRY(hipGetLastError());
    return LIRA_OK;
}

}  // extern "C"
