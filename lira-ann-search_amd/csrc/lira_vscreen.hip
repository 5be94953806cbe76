// lira_vscreen.hip -- the wave-resident screen k_screen_v (gfx950): every wave
// is its own work item (64 query rows x one chunk of a bucket), the rows' hi
// parts of fl(q - c) sit in registers for the whole item, the candidates' hi
// parts are loaded straight from Xb into registers (two tiles in flight), and
// v_mfma_f32_16x16x32_bf16 screens 64 rows x 64 candidates per tile.  No LDS
// staging, no workgroup barrier: the four waves of a workgroup never wait for
// each other.  LDS holds only each wave's row lists and survivor buffers.
//
// Replaces search.cpp:468-493 (the per-query candidate loop over the probed
// buckets) for L2 with the centred split copy, k <= 24, dpad 64 / 96 / 128;
// results identical to the all-exact scan.  The error model and the fp32 bound
// arithmetic are k_screen_w's (lira_wscreen.hip: werr_E, bndP, the skip
// interval), which are k_screen_m<..., 3>'s (lira_bounds.hpp err_E, split 3)
// rounded outward.
//
// Why.  k_screen_m (4 waves share an LDS-staged block of 256 candidates) spends
// ~16.7 k cycles per block on SIFT1M mixture against ~1 k of MFMA work: every
// chunk is a DMA issue, a counted wait and a workgroup barrier, and each wave
// re-reads the whole staged block from LDS (phase clocks,
// profiles/r03_sift1m_*_phase_clocks.txt).  Here a tile costs 17 global loads
// per lane, 64 MFMAs and the selection, all within one wave.
//
// Row lists: a row's survivors are appended to its 32-key buffer; a full
// buffer is merged into the row's sorted 32-key list (half-wave network).  At
// the item's end a row whose list is still empty and whose buffer is not full
// is written out UNSORTED (its keys, then empty keys): k_smerge walks such
// lists to the first empty key (SMergeArgs::unsorted) -- the merge of every
// row's buffer at every item end is what made k_screen_m's epilogue ~8 % of its
// cycles.  Rows whose list filled are merged and written sorted as before.
#include <algorithm>
#include <atomic>
#include <string>

#include "lira_bounds.hpp"
#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

typedef __bf16 vbf16x8 __attribute__((ext_vector_type(8)));
typedef float vf4 __attribute__((ext_vector_type(4)));

static constexpr int kVRT = 2;      // row tiles of 16 per wave
static constexpr int kVQR = 16 * kVRT;  // query rows per item (one wave): 32
static constexpr int kVW = 4;       // independent waves per workgroup
static constexpr int kVOcc = 2;     // workgroups per CU (2 waves per SIMD: <= 256 registers per wave)
static constexpr int kVK2 = 32;     // row list keys (k <= 24)
static constexpr int kVBC = 32;     // survivor buffer keys per row
static constexpr int kVMaxT = 128;  // tiles per item (their radius ranges: 2 registers per lane)

struct VSmem {  // per wave
    static constexpr int lists = 0;                            // [QR][K2] u64
    static constexpr int bufs = lists + kVQR * kVK2 * 8;       // [QR][BC] u64
    static constexpr int kth = bufs + kVQR * kVBC * 8;         // [QR] u64: list key k - 1
    static constexpr int hs = kth + kVQR * 8;                  // [QR] f32: the rows' dot thresholds
    static constexpr int qns = hs + kVQR * 4;                  // [QR] f32: the rows' fl(||q'||^2)
    static constexpr int bcs = qns + kVQR * 4;                 // [QR] int: buffer fills
    static constexpr int rq = bcs + kVQR * 4;                  // [QR] float4: qn, qnorm, dq, qres of the row
    static constexpr int tr = rq + kVQR * 16;                  // [kVMaxT] float4: tile lo, hi, hi residual
    static constexpr int per_wave = tr + kVMaxT * 16;
    static constexpr int total = kVW * per_wave;
};
static_assert(VSmem::total * kVOcc <= 160 * 1024, "k_screen_v LDS");

struct VArgs {
    const uint16_t *Xb;
    const float *xadj;   // centred (xadjc)
    const int32_t *qlist;
    const int4 *vrec;    // k_vrec's per-item records, 2 int4 each
    int32_t *head;
    const float *Q, *pivot;
    const float4 *QN;    // per pair: qn, qnorm (up), -, ||q - c|| (k_pairs)
    const float *QE;     // per pair: ||q' - hi(q')|| (up)
    const uint16_t *QH;  // per pair: hi(fl(q - c)) bf16, dpad dims (k_pairs; zero past d)
    const float2 *tstat;
    const float *tres;
    u64 *partial;
    float *pE;
    uint32_t *qbound;
    int64_t d, dpad;
    int nprobe, k, nch_max, share, tri;
    unsigned long long *stats;
};

// ---- per-item records (one thread per item of k_plan's table) ----
// 0 p, 1 chunk, 2 first pair index into qlist, 3 rows; 4 first tile (absolute),
// 5 tiles, 6 rmax bits (centred)
__global__ __launch_bounds__(256) void k_vrec(const int4 *itab, const int32_t *head, const int32_t *tile_off,
                                              const int32_t *qoff, const int32_t *cnt, const float *rmax,
                                              int n_lists, int n_virt, int bpc, int bpc_near, int4 *vrec) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= head[18]) return;
    const int4 e = itab[i];
    const int vp = e.x, qb = e.y, ch = e.z;
    const int p = vp >= n_lists ? vp - n_lists : vp;
    const int tile0 = tile_off[p], ntl = tile_off[p + 1] - tile0;
    const int b = vp < n_lists && n_virt > n_lists ? bpc_near : bpc;
    const int tbb = ch * b * 4, tbe = min(ntl, tbb + b * 4);
    vrec[2 * i] = make_int4(p, ch, qoff[vp] + qb * kVQR, min(kVQR, cnt[vp] - qb * kVQR));
    vrec[2 * i + 1] = make_int4(tile0 + tbb, tbe - tbb, __float_as_int(rmax[p]), 0);
}

// fp32 bound arithmetic of k_screen_w (lira_wscreen.hip), rounded outward
__device__ __forceinline__ float vup(float x) { return __builtin_fmaf(__builtin_fabsf(x), 0x1p-22f, x); }
__device__ __forceinline__ float vdn(float x) { return __builtin_fmaf(-__builtin_fabsf(x), 0x1p-22f, x); }
__device__ __forceinline__ float verr_E(float qnorm, float Rb, float dpf, float hres, float qres) {
    const float ex = hres >= 0.0f ? hres * 1.0002f : 0x1p-8f * 1.03f * Rb;
    const float re = Rb + ex;
    const float ed = ex * qnorm + qres * re * 1.0002f + 2.0f * dpf * 0x1p-22f * 1.03f * qnorm * re +
                     2.0f * dpf * 0x1p-96f * (qnorm + re + 1.0f);
    const float s = qnorm + Rb;
    return vup((2.0f * ed + 10.5f * 0x1p-24f * s * s + 0x1p-126f) * (1.0f + 0x1p-17f));
}
__device__ __forceinline__ int vxcd_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 7u);
}
__device__ __forceinline__ int vrow16_incl_scan(int v) {  // within each 16-lane DPP row
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    return v;
}
__device__ __forceinline__ int vrow16_total(int inc) {
    const int t0 = __builtin_amdgcn_readlane(inc, 15), t1 = __builtin_amdgcn_readlane(inc, 31);
    const int t2 = __builtin_amdgcn_readlane(inc, 47), t3 = __builtin_amdgcn_readlane(inc, 63);
    const int g = (int)(threadIdx.x & 63) >> 4;
    return g == 0 ? t0 : g == 1 ? t1 : g == 2 ? t2 : t3;
}
__device__ __forceinline__ float vlane(float v, int l) {  // uniform lane index
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

#ifdef LIRA_VCLOCKS
static constexpr bool kVClk = true;  // timing build: phase cycles of wave 0 into the stats words
#else
static constexpr bool kVClk = false;
#endif

template <int NKS>
__global__ __launch_bounds__(64 * kVW, kVOcc) void k_screen_v(VArgs a) {
    constexpr int RT = kVRT, QR = kVQR;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int g = lane >> 4, cj = lane & 15;
    char *const wsm = smem + wave * VSmem::per_wave;
    u64 *const lists = (u64 *)(wsm + VSmem::lists);
    u64 *const bufs = (u64 *)(wsm + VSmem::bufs);
    u64 *const kth_s = (u64 *)(wsm + VSmem::kth);
    float *const h_s = (float *)(wsm + VSmem::hs);
    float *const qn_s = (float *)(wsm + VSmem::qns);
    int *const bc_s = (int *)(wsm + VSmem::bcs);
    float4 *const tr_s = (float4 *)(wsm + VSmem::tr);
    float4 *const rq_s = (float4 *)(wsm + VSmem::rq);
    const int k = a.k;
    const double dd = (double)a.d;
    unsigned long long *const cnt = kVClk ? nullptr : a.stats;
    long long ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t1c = 0;
    auto tick = [&](int s) {
        if (kVClk) {
            const long long t = clock64();
            ck[s] += t - t1c;
            t1c = t;
        }
    };
    // bound_P's factor (1 + (d+4) u)(1 + 2^-50) and 1 / F, F = 1 - (d+4) u, rounded up
    const float Gp = __double2float_ru((1.0 + (dd + 4.0) * kU) * (1.0 + 0x1p-40));
    const float iF = __double2float_ru((1.0 / (1.0 - (dd + 4.0) * kU)) * (1.0 + 0x1p-40));
    const float dpf = (float)a.dpad;
    auto bndP = [&](float sk, float E) { return vup(vup(vup(sk + E) * Gp) + 0x1p-126f); };
    const int nkc = (int)(a.dpad / 16);  // 16-dim chunks of a tile in Xb (4 KiB each)

    // ---- items: lane 0 claims from its XCD's queue (k_plan), stealing when empty;
    // the next claim's atomic is issued one item ahead and resolved at the next item
    int qx = vxcd_id(), tries = 0;
    auto claim_issue = [&]() -> int {
        int raw = 0;
        if (lane == 0 && tries < 8) raw = a.head[10 + qx] + atomicAdd(&a.head[2 + qx], 1);
        return raw;
    };
    auto claim_resolve = [&](int raw) -> int {
        int it = -1;
        if (lane == 0) {
            int i = raw;
            while (tries < 8) {
                if (i < a.head[11 + qx]) {
                    it = i;
                    break;
                }
                qx = (qx + 1) & 7;
                if (++tries >= 8) break;
                i = a.head[10 + qx] + atomicAdd(&a.head[2 + qx], 1);
            }
        }
        return __builtin_amdgcn_readfirstlane(it);
    };

    // half-wave merge of a row's buffer (n keys) into its sorted list; the
    // list's key k - 1 is kept in kth_s for the refresh (lane = row reads it
    // without the 64-way bank conflict of a strided list read)
    auto flush1 = [&](int row, int n) {
        const int hl = lane & 31;
        u64 lst[1] = {lists[row * kVK2 + hl]};
        const u64 b = hl < n ? bufs[row * kVBC + hl] : kEmptyKey;
        half_merge_batch1<1>(lst, b);
        if (lane < 32) lists[row * kVK2 + hl] = lst[0];
        if (lane == k - 1) kth_s[row] = lst[0];
        __builtin_amdgcn_wave_barrier();
    };
    auto flush2 = [&](int ra, int na, int rb, int nb) {  // two rows, one per half-wave
        const int hl = lane & 31;
        const int row = lane < 32 ? ra : rb, n = lane < 32 ? na : nb;
        u64 lst[1] = {lists[row * kVK2 + hl]};
        const u64 b = hl < n ? bufs[row * kVBC + hl] : kEmptyKey;
        half_merge_batch1<1>(lst, b);
        lists[row * kVK2 + hl] = lst[0];
        if (hl == k - 1) kth_s[row] = lst[0];
        __builtin_amdgcn_wave_barrier();
    };

    int raw_next = claim_issue();
    if (kVClk) t1c = clock64();
#pragma unroll 1
    for (;;) {
        const int it = claim_resolve(raw_next);
        tick(7);
        if (it < 0) break;
        raw_next = claim_issue();
        const int4 r0 = a.vrec[2 * it], r1 = a.vrec[2 * it + 1];
        const int p = __builtin_amdgcn_readfirstlane(r0.x), ch = __builtin_amdgcn_readfirstlane(r0.y);
        const int pbase = __builtin_amdgcn_readfirstlane(r0.z), nval = __builtin_amdgcn_readfirstlane(r0.w);
        const int tfirst = __builtin_amdgcn_readfirstlane(r1.x), ntiles = __builtin_amdgcn_readfirstlane(r1.y);
        const float R = __int_as_float(__builtin_amdgcn_readfirstlane(r1.z));

        // ---- rows: lane = row
        const int my_pair = lane < nval && lane < QR ? a.qlist[pbase + lane] : -1;
        const int my_q = my_pair >= 0 ? my_pair / a.nprobe : -1;
        float4 qr = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float my_qres = 0.0f;
        uint32_t pub = ~0u;
        if (my_pair >= 0) {
            qr = a.QN[my_pair];
            my_qres = a.QE[my_pair];
            if (a.qbound) pub = __hip_atomic_load(a.qbound + my_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // (the row's constants live in LDS between refreshes: registers are short at
        // 2 waves per SIMD, and a spill reload in the tile loop would drain vmcnt)
        if (lane < QR) {
            rq_s[lane] = make_float4(qr.x, qr.y, qr.w, my_qres);
            qn_s[lane] = qr.x;
            bc_s[lane] = 0;
            kth_s[lane] = kEmptyKey;
        }
        {
            uint4 *L4 = (uint4 *)lists;
#pragma unroll
            for (int i = 0; i < QR * kVK2 / 2 / 64; ++i) L4[i * 64 + lane] = make_uint4(~0u, ~0u, ~0u, ~0u);
        }
        // ---- the rows' hi parts of fl(q - c): A fragments (lane (g, cj): row 16 rt + cj,
        // dims 32 s + 8 g .. + 7)
        vbf16x8 Aq[RT][NKS];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int pr = __shfl(my_pair, rt * 16 + cj, 64);
            const vbf16x8 *qh = (const vbf16x8 *)(a.QH + (int64_t)(pr >= 0 ? pr : 0) * a.dpad + 8 * g);
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                const vbf16x8 v = qh[4 * s];  // (branch-free: row 0's, then zeroed for an empty row)
                Aq[rt][s] = pr >= 0 ? v : (vbf16x8)(__bf16)0.0f;
            }
        }
        // ---- the item's tile radius ranges / hi residuals into LDS (tr_s[t])
#pragma unroll
        for (int u = 0; u < kVMaxT / 64; ++u) {
            const int t = lane + 64 * u;
            float lo = -__builtin_inff(), hi = __builtin_inff(), re = -1.0f;
            if (t < ntiles) {
                if (a.tri) {
                    const float2 st = a.tstat[tfirst + t];
                    lo = st.x;
                    hi = st.y;
                }
                if (a.tres) re = a.tres[tfirst + t];
            }
            tr_s[t] = make_float4(lo, hi, re, 0.0f);
        }
        __builtin_amdgcn_wave_barrier();
        // ---- row threshold state (lane = row)
        float E_run = 0.0f, T_c = -1.0f, A_c = 0.0f, h_l = 0.0f;
        uint32_t own_pub = ~0u;
        float2 ab_c;
        auto interval = [&](float T, float my_dq) {  // the row's skip interval for ||x - c|| under bound T (+ A_c)
            float2 ab = make_float2(-__builtin_inff(), __builtin_inff());
            A_c = vup(vup(fmaxf(T, 0.0f) + 0x1p-126f) * iF);
            if (my_pair < 0) {
                ab = make_float2(__builtin_inff(), -__builtin_inff());
            } else if (T < 3e38f && iF < 2.0f) {
                const float rad = vup(vup(sqrtf(A_c)) * (1.0f + 0x1p-20f));
                ab = make_float2(vdn(vdn(my_dq * (1.0f - 0x1p-21f)) - rad), vup(vup(my_dq * (1.0f + 0x1p-21f)) + rad));
            }
            return ab;
        };
        ab_c = interval(pub != ~0u ? ord2f(pub) : __builtin_inff(), qr.w);
        const bool any_row = __any(my_pair >= 0);
        // first tile >= t that some row may need (current intervals; stale ones are wider: safe)
        auto next_live = [&](int t) {
            if (!a.tri) return t;
            while (t < ntiles) {
                const float4 tv = tr_s[t];  // (uniform address: one broadcast read)
                const float lo = tv.x, hi = tv.y;
                if (!__all(hi < ab_c.x || lo > ab_c.y)) break;
                ++t;
            }
            return t;
        };
        tick(1);

        // ---- x fragments of tile t into buffer B (lane (g, cj): dims 32 s + 8 g .. of
        // candidate 4 cj + ct, Xb piece (2 s + (g >> 1), hi part g & 1), p = 16 ct + cj)
        vbf16x8 B0[NKS][4], B1[NKS][4];
        vf4 xa0, xa1;
        // buffer loads off one per-item resource: a single VGPR offset per lane and
        // scalar offsets per piece (flat addresses needed a 64-bit VGPR pair per 4 KiB
        // of immediate-offset reach, which spilled at 2 waves per SIMD)
        const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.Xb + (int64_t)tfirst * nkc * 2048), (short)0, ntiles * nkc * 4096, 0x00020000);
        const int voff = (g >> 1) * 4096 + (g & 1) * 1024 + cj * 16;
        auto issue = [&](vbf16x8 (&B)[NKS][4], vf4 &xa, int t) {
            const int tc = min(t, ntiles - 1);  // (past the end: a valid tile, not used)
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int ct = 0; ct < 4; ++ct)
                    B[s][ct] = __builtin_bit_cast(
                        vbf16x8, __builtin_amdgcn_raw_buffer_load_b128(xrs, voff, tc * nkc * 4096 + s * 8192 + ct * 256, 0));
            xa = *(const vf4 *)(a.xadj + (int64_t)(tfirst + tc) * kTile + 4 * cj);
        };

        uint32_t pub_next = pub;
        const int my_qs = my_q >= 0 ? my_q : 0;  // (qbound is non-null here: the seeded bound)
        // ---- one tile: refresh the rows' thresholds, MFMAs, selection
        auto process = [&](const vbf16x8 (&B)[NKS][4], const vf4 &xa, int t) {
            // refresh (lane = row)
            const float4 tv = tr_s[t];
            const float b_lo = tv.x, b_hi = tv.y, b_re = tv.z;
            const u64 kk = lane < QR ? kth_s[lane] : kEmptyKey;
            float T = kk == kEmptyKey ? __builtin_inff() : bndP(key_score(kk), E_run);
            if (a.share) {
                if (my_pair >= 0 && kk != kEmptyKey) {
                    const uint32_t b = f2ord(T);
                    if (b < own_pub) {
                        atomicMin(a.qbound + my_q, b);
                        own_pub = b;
                    }
                }
                // the query's bound as published before this tile (loaded one tile
                // ahead, unconditionally: its wait then covers only older loads)
                pub = my_pair >= 0 ? min(pub, pub_next) : pub;
                pub_next = __hip_atomic_load(a.qbound + my_qs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (pub != ~0u) T = fminf(T, ord2f(pub));
            const float4 rq = lane < QR ? rq_s[lane] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            const float my_qn = rq.x, my_qnorm = rq.y, my_qres = rq.w;
            if (T != T_c) {
                T_c = T;
                ab_c = interval(T, rq.z);
            }
            const float Rb = a.tri ? fminf(R, vup(b_hi * (1.0f + 0x1p-19f))) : R;
            const float Eb = verr_E(my_qnorm, Rb, dpf, b_re, my_qres);
            const float lim = vup(A_c + Eb);
            const float sq = vup((my_qnorm + Rb) * (my_qnorm + Rb));
            const float c = vup(1.06f * 0x1p-24f * sq);
            const float h0 = (my_qn - lim) * 0.5f - c;
            h_l = my_pair < 0 ? __builtin_inff() : h0 - (__builtin_fabsf(my_qn) + lim + c) * 0x1p-21f;
            const bool wdead = !any_row || (a.tri && __all(b_hi < ab_c.x || b_lo > ab_c.y));
            if (cnt && lane == 0) {
                atomicAdd(cnt + 2, 1ull);
                if (!wdead) atomicAdd(cnt + 0, 64ull * kTile);
            }
            tick(2);
            if (wdead) return;
            E_run = fmaxf(E_run, Eb);  // (this tile's keys may join the lists)
            if (lane < QR) h_s[lane] = h_l;
            __builtin_amdgcn_wave_barrier();
            vf4 hp[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const vf4 h4 = *(const vf4 *)(h_s + rt * 16 + 4 * g);
                // (padding: xadj = +inf gives -inf, which never passes a finite threshold)
#pragma unroll
                for (int r = 0; r < 4; ++r) hp[rt][r] = fmaxf(h4[r], -3.40282347e38f);
            }
            // MFMAs: 4 row tiles x 4 candidate groups x NKS k-steps
            vf4 acc[RT][4];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int ct = 0; ct < 4; ++ct) acc[rt][ct] = (vf4)(0.0f);
#ifdef LIRA_VDBG
            if (!(LIRA_VDBG & 2))
#endif
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int ct = 0; ct < 4; ++ct)
                        acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Aq[rt][s], B[s][ct], acc[rt][ct], 0, 0, 0);
            tick(3);
#ifdef LIRA_VDBG  // timing experiments (results invalid): 1 = no selection, 2 = no MFMA either
            if (LIRA_VDBG & 1) {
                float z = 0.0f;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int ct = 0; ct < 4; ++ct) z += (LIRA_VDBG & 2) ? (float)B[0][ct][rt] : acc[rt][ct][0];
                if (z == 1234.5f) bufs[lane] = 1;
                return;
            }
#endif
            // selection: lane (g, cj) holds rows 16 rt + 4 g + r, candidates 4 cj + ct
            float m[RT][4];
            bool anyp = false;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float w0 = acc[rt][0][r] - xa[0], w1 = acc[rt][1][r] - xa[1];
                    const float w2 = acc[rt][2][r] - xa[2], w3 = acc[rt][3][r] - xa[3];
                    m[rt][r] = fmaxf(fmaxf(w0, w1), fmaxf(w2, w3));
                    anyp |= m[rt][r] >= hp[rt][r];
                }
            if (!__any(anyp)) {
                tick(4);
                return;
            }
            const uint32_t tid0 = (uint32_t)(tfirst + t) * kTile + 4 * cj;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (!__any(m[rt][r] >= hp[rt][r])) continue;
                    const float h = hp[rt][r];
                    int pm = 0;
#pragma unroll
                    for (int ct = 0; ct < 4; ++ct) pm |= (acc[rt][ct][r] - xa[ct] >= h) << ct;
                    const int row = rt * 16 + 4 * g + r;
                    const int n_l = __builtin_popcount(pm);
                    const int inc = vrow16_incl_scan(n_l);
                    const int tot = vrow16_total(inc);  // (group-uniform: the row's new keys)
                    const int bc0 = bc_s[row];
                    const bool pre = bc0 > 0 && bc0 + tot > kVBC;  // merge the buffer first
                    const int total = (pre ? 0 : bc0) + tot;
                    const int base = (pre ? 0 : bc0) + inc - n_l;
                    const float qn_r = qn_s[row];
                    for (int w0 = 0;; w0 += kVBC) {
                        u64 fl = __ballot((w0 == 0 ? pre : total > w0) && cj == 0);
                        while (fl) {
                            const int gg = __builtin_ctzll(fl) >> 4;
                            fl &= fl - 1;
                            flush1(rt * 16 + 4 * gg + r, w0 == 0 ? __builtin_amdgcn_readlane(bc0, 16 * gg) : kVBC);
                        }
                        int rank = base;
#pragma unroll
                        for (int ct = 0; ct < 4; ++ct) {
                            if ((pm >> ct) & 1) {
                                if (rank >= w0 && rank < w0 + kVBC) {
                                    const float sc = __builtin_fmaf(-2.0f, acc[rt][ct][r], qn_r + 2.0f * xa[ct]);
                                    bufs[row * kVBC + rank - w0] = ((u64)f2ord(sc) << 32) | (tid0 + (uint32_t)ct);
                                }
                                ++rank;
                            }
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (!__any(total - w0 > kVBC)) break;
                    }
                    if (cj == 0) bc_s[row] = total <= kVBC ? total : total - kVBC * ((total - 1) / kVBC);
                    if (cnt && cj == 0 && tot) atomicAdd(cnt + 7, (unsigned long long)tot);
                    __builtin_amdgcn_wave_barrier();
                }
            tick(4);
        };

        // ---- the tile loop: two register buffers, the next tile's loads in flight
        // under this tile's work
        int ta = next_live(0);
        if (ta < ntiles) {
            issue(B0, xa0, ta);
            int tb = next_live(ta + 1);
            issue(B1, xa1, tb);
#pragma unroll 1
            for (;;) {
                process(B0, xa0, ta);
                if (tb >= ntiles) break;
                ta = next_live(tb + 1);
                issue(B0, xa0, ta);  // (unconditional: past the end it loads a valid tile, unused --
                                     // a conditional load would make hipcc's vmcnt counts conservative)
                tick(5);
                process(B1, xa1, tb);
                if (ta >= ntiles) break;
                tb = next_live(ta + 1);
                issue(B1, xa1, tb);
                tick(5);
            }
        }

        // ---- epilogue: merge the rows whose lists filled; lists out (two rows per round)
        const int bcl = lane < QR ? bc_s[lane] : 0;
        const bool srt = lane < QR && (kth_s[lane] != kEmptyKey || lists[lane * kVK2] != kEmptyKey || bcl == kVBC);
        {
            u64 mrg = __ballot(bcl > 0 && srt);
            while (mrg) {
                const int ra = __builtin_ctzll(mrg);
                mrg &= mrg - 1;
                int rb = ra;
                if (mrg) {
                    rb = __builtin_ctzll(mrg);
                    mrg &= mrg - 1;
                }
                const int na = __builtin_amdgcn_readlane(bcl, ra), nb = __builtin_amdgcn_readlane(bcl, rb);
                if (rb != ra) flush2(ra, na, rb, nb);
                else flush1(ra, na);
            }
        }
        const u64 srt_m = __ballot(srt);
        const int hl = lane & 31;
#pragma unroll 1
        for (int r2 = 0; r2 < QR; r2 += 2) {
            const int row = r2 + (lane >> 5);
            const int pr = __shfl(my_pair, row, 64);
            const int nb = __shfl(bcl, row, 64);
            if (pr >= 0) {
                const u64 v = ((srt_m >> row) & 1) ? lists[row * kVK2 + hl] : hl < nb ? bufs[row * kVBC + hl] : kEmptyKey;
                a.partial[((int64_t)pr * a.nch_max + ch) * kVK2 + hl] = v;
            }
        }
        if (my_pair >= 0) {
            if (a.pE) a.pE[(int64_t)my_pair * a.nch_max + ch] = fmaxf(E_run, 0x1p-126f);
            const u64 kk = kth_s[lane];
            if (a.qbound && kk != kEmptyKey) atomicMin(a.qbound + my_q, f2ord(bndP(key_score(kk), E_run)));
        }
        __builtin_amdgcn_wave_barrier();
        tick(6);
    }
    if (kVClk && a.stats && lane == 0 && wave == 0) {
        // [1] item prologue, [2] refresh, [3] MFMA issue, [4] selection, [5] issue + skip, [6] epilogue,
        // [7] claims
        for (int i = 1; i < 8; ++i) atomicAdd(a.stats + i, (unsigned long long)ck[i]);
    }
}

// ------------------------------------------------------------------ host side
template <int NKS>
static hipError_t launch_v(const VArgs &a, int grid, hipStream_t st) {
    static std::atomic<uint64_t> attr{0};
    hipError_t e = set_smem_attr_once(attr, (const void *)k_screen_v<NKS>, VSmem::total);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_screen_v<NKS>), dim3(grid * kVOcc), dim3(64 * kVW), VSmem::total, st, a);
    return hipGetLastError();
}

bool vscreen_shape_ok(int64_t dpad) { return dpad == 64 || dpad == 96 || dpad == 128; }
int vscreen_smem() { return VSmem::total; }
int vscreen_max_tiles() { return kVMaxT; }
int vscreen_rows() { return kVQR; }
int vscreen_workers_per_cu() { return kVW * kVOcc; }

hipError_t launch_vscreen(const lira_index *idx, const float *q, const int32_t *cnt, const int32_t *qoff,
                          const int32_t *qlist, const int4 *itab, int32_t *head, const float4 *QN, const float *QE,
                          const uint16_t *QH, u64 *partial, float *pE, uint32_t *qbound, int nprobe, int k, int bpc,
                          int bpc_near, int nch_max, int n_virt, int tri, int grid, int4 *vrec, int64_t max_items,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_vrec, dim3((unsigned)((max_items + 255) / 256)), dim3(256), 0, st, itab, head, idx->tile_off,
                       qoff, cnt, idx->rmaxc, (int)idx->n_lists, n_virt, bpc, bpc_near, vrec);
    VArgs a;
    a.Xb = idx->Xb;
    a.xadj = idx->xadjc;
    a.qlist = qlist;
    a.vrec = vrec;
    a.head = head;
    a.Q = q;
    a.pivot = idx->pivot;
    a.QN = QN;
    a.QE = QE;
    a.QH = QH;
    a.tstat = idx->tstat;
    a.tres = idx->tres;
    a.partial = partial;
    a.pE = pE;
    a.qbound = qbound;
    a.d = idx->d;
    a.dpad = idx->dpad;
    a.nprobe = nprobe;
    a.k = k;
    a.nch_max = nch_max;
    a.share = idx->opt.share;
    a.tri = tri && idx->tstat != nullptr;
    a.stats = idx->stats_on ? (unsigned long long *)idx->stats : nullptr;
    switch (idx->dpad) {
        case 64: return launch_v<2>(a, grid, st);
        case 96: return launch_v<3>(a, grid, st);
        case 128: return launch_v<4>(a, grid, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace lira
