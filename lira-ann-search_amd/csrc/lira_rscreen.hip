// lira_rscreen.hip -- k_screen_r, the wave-streaming screen (gfx950): the
// default screen of lira_scan_topk for L2 and for IP on a centred index
// (lira_index::ipc), k <= 120, dpad <= 128.  Replaces search.cpp:468-493 (the
// per-query loop over the candidates of the probed buckets, l2_sq :253-260 /
// -ip :263-269) with results identical to the all-exact scan: it screens every
// (query, candidate) pair with a rigorous bound and leaves the exact re-check
// and the top-k to k_smerge (lira_screen.hip), exactly as k_screen_m does.  The
// error model is k_screen_m<..., 3>'s (hi x hi, lira_bounds.hpp err_E, split =
// 3), evaluated in fp32 with explicit outward rounding.
//
// Work split.  An item is (bucket, block of QR query rows, chunk of the bucket):
//   * the item's QR query rows' hi parts live in LDS in MFMA-fragment order (the
//     A operands, loaded once per item from the per-pair records of k_seed_t /
//     k_pairs);
//   * each of the 4 waves streams its OWN candidate tiles (64 rows each; tiles
//     u, u + 4, ... of the item): B fragments straight from HBM/L2 into
//     registers, one 16-B load per lane feeding QR/16 MFMAs, the next tile's
//     loads issued under the current tile's MFMAs -- no LDS staging of
//     candidates, no barrier inside an item;
//   * the four waves share the item's QR row lists (LDS, sorted, K2 = 32 RL
//     keys); each wave appends survivors to its own per-row buffers (16 keys)
//     and merges a full buffer into the shared list under a per-row LDS lock;
//     thresholds follow the shared lists, the per-row error bound and the
//     query's published bound.
// RL = 1 (k <= 24): 64 query rows per item, 32-key lists.  RL = 2 / 4 (k <= 56 /
// 120, DEEP10M's k = 100): 32 rows per item, 64 / 128-key lists, so that the
// lists, buffers and A operands stay within 80 KB of LDS (two workgroups per
// CU; the MFMA count per pair is the same, each candidate byte feeds 32 rows
// instead of 64).
//
// Metrics.  L2: x' = fl(x - c), q' = fl(q - c) for the list pivot c; score s~ =
// fl(qn - 2 fl(dot' - xadj)), qn = fl(||q'||^2), xadj = fl(||x'||^2)/2; block skip
// by the triangle inequality.  IP (centred): q stays, x' = fl(x - c), and q.x
// = q.x' + q.c, so s~ = -fl(dot' + qc), qc = fl(q.c) per (query, list) pair;
// block skip by Cauchy-Schwarz, -q.x >= -q.c - ||q|| ||x - c||.
//
// MFMA layout (cdna_hip_programming.md, 16x16x32 bf16): A = 16 query rows x
// 32 dims (lane l: row l & 15, dims 8 (l >> 4) ..), B = 32 dims x 16
// candidates (lane l: candidate slot l & 15 of group i, the same dims), read
// from Xb's hi quarters: 16-dim chunk 2c + (g >> 1), part g & 1, slot 16 i +
// (l & 15) = storage row 4 (l & 15) + i of the tile.  D: lane (g, j) holds
// rows 4 g + reg of the row group, candidate 4 j + i.
#include <atomic>

#include "lira_bounds.hpp"
#include "lira_internal.hpp"
#include "lira_rscreen.hpp"

namespace lira {

typedef __bf16 rbf16x8 __attribute__((ext_vector_type(8)));
typedef float rf4 __attribute__((ext_vector_type(4)));

static constexpr int kRMaxTiles = 512;  // tiles per item (the plan caps a chunk at 128 blocks)
static constexpr int kROCap = 128;      // survivor queue entries per wave (>= two candidate masks)

// W waves per workgroup (an item): 4 (two workgroups per CU) or 8 (one, with QR = 64
// rows at RL 4: the 128-key lists of 64 rows and 8 waves' buffers in one CU's LDS)
template <int RL, int W>
struct RSmem {
    static constexpr int QR = RL == 1 || W == 8 ? 64 : 32;         // query rows per item
    static constexpr int K2 = 32 * RL;                             // row list keys
    static constexpr int NRG = QR / 16;                            // MFMA row groups
    // survivor buffer keys per (wave, row): as many as the 80 KB allow -- every full
    // buffer costs a locked 32 RL-key list merge (DEEP10M mixture, RL 4: 16 -> 24
    // keys, scan 2.82 -> 2.17 ms); 6 bytes a key: its high word and its position in
    // the item (the list key is rebuilt when merged)
    static constexpr int BC = W == 8 ? 8 : RL == 1 ? 21 : 32;  // (<= 32: a flush merges one key per half-wave lane)
    // buffer strides in entries: odd per row (BCS) and per wave (WS = 1 mod 32), so the
    // lanes of a drain round that write the same slot of different rows, and the
    // epilogue's reads of the same slot of different waves' buffers, fall on
    // different banks (a 32-entry row stride put every row's slot s on one bank)
    static constexpr int BCS = BC | 1;
    static constexpr int WS = QR * BCS + ((1 - QR * BCS) & 31);
    static constexpr int aq = 0;                                   // [4 chunks][NRG][64 lanes] 16 B: A operands
    static constexpr int lists = aq + 4 * NRG * 64 * 16;           // [QR][K2] u64
    static constexpr int bufs = lists + QR * K2 * 8;               // [W][WS] u32: [row][BCS] wkey high words
    static constexpr int bufl = bufs + W * WS * 4;                 // [W][WS] u16: positions in the item
    static constexpr int bufc = (bufl + W * WS * 2 + 15) & ~15;    // [W][64] int (lane = row)
    static constexpr int hs = bufc + W * 64 * 4;                   // [W][64] float: the wave's thresholds
    static constexpr int tst = hs + W * 64 * 4;                    // [512] float2: tile radius ranges
    static constexpr int trs = tst + kRMaxTiles * 8;               // [512] float: tile hi residuals
    static constexpr int pair = trs + kRMaxTiles * 4;              // [64] int
    static constexpr int qn = pair + 64 * 4;                       // [64] float4: qn (IP qc), ||q'|| (up), qres, dq (IP qc)
    static constexpr int erun = qn + 64 * 16;                      // [64] float bits: running error bound
    static constexpr int lock = erun + 64 * 4;                     // [64] int
    static constexpr int opub = lock + 64 * 4;                     // [64] uint: bound last published
    static constexpr int oqk = opub + 64 * 4;                      // [W][kROCap] u64: survivor queue keys
    static constexpr int kth = oqk + W * kROCap * 8;               // [64] u64: each list's k-th key
    static constexpr int meta = kth + 64 * 8;                      // [16] int
    static constexpr int total = meta + 64;
};
static_assert(RSmem<1, 4>::total <= 80 * 1024 && RSmem<2, 4>::total <= 80 * 1024 && RSmem<4, 4>::total <= 80 * 1024,
              "k_screen_r: two 4-wave workgroups per CU");
static_assert(RSmem<4, 8>::total <= 160 * 1024, "k_screen_r: one 8-wave workgroup per CU");
static_assert(RSmem<1, 4>::BC <= 32 && RSmem<2, 4>::BC <= 32 && RSmem<4, 4>::BC <= 32, "flush_row merges <= 32 keys");
static_assert(kROCap >= 128, "a drained queue takes two full candidate masks");

// a value the compiler must treat as produced here (keeps per-lane address
// arithmetic from being hoisted out of the loops: hipcc otherwise precomputed
// ~80 VGPRs of row addresses for the 16 selection entries)
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// outward rounding by a margin covering a handful of fp32 roundings
__device__ __forceinline__ float rup(float x) { return __builtin_fmaf(__builtin_fabsf(x), 0x1p-20f, x) + 0x1p-125f; }
__device__ __forceinline__ float rdn(float x) { return __builtin_fmaf(-__builtin_fabsf(x), 0x1p-20f, x) - 0x1p-125f; }

// err_E(qnorm, Rb, d, split = 3, dpad, centred, hres, qres) in fp32: every term is
// >= 0, so the ~16 roundings stay below 2^-20 relative and the final factor covers
// them; + 2^-125 >= d 2^-140 (lira_bounds.hpp).
// The MFMA chain starts from C = -xadj (no separate fl(dot - xadj)): one more
// add, and every partial sum is bounded by xadj + ||q'|| (R + rho), xadj <=
// fl(Rb^2) / 2 (L2; 0 for IP), so the accumulation term counts dpad + 1 adds at
// 2^-22 of that (lira_bounds.hpp's model: any order or rounding mode at <= 2^-22
// per add).
// L2: E = 2 ed + (8.4 + 2.01 + 2) u (||q'|| + Rb)^2 (the centred copy's 2.01 u s^2,
// s~ = fl(qn - 2 wv)'s extra rounding 2 u s^2).
// IP (centred): s~ = -fl(wv + qc) against search.cpp's s = -fl_seq(q.x):
//   |q.x' - wv| <= ed;  |q.(x - c - x')| <= 1.01 u ||q|| Rb (x' = fl(x - c));
//   |qc - q.c| <= 1.01 u |qc|;  the add: u (||q|| (Rb + rho) + |qc|);
//   search.cpp's own sum: (d + 2) u ||q|| Rx, Rx >= ||x|| (the list's rmax).
template <int M>
__device__ __forceinline__ float errE_r(float qnorm, float Rb, float hres, float qres, float dp, float qc, float Rx,
                                        float dd) {
    const float ex = hres >= 0.0f ? hres * 1.0001f : 0x1p-8f * 1.02f * Rb;
    const float xa = M == LIRA_METRIC_L2 ? 0.5001f * Rb * Rb : 0.0f;
    const float ed = ex * qnorm + qres * (Rb + ex) * 1.0001f + 2.0f * (dp + 1.0f) * 0x1p-22f * 1.02f * (qnorm * (Rb + ex) + xa) +
                     2.0f * dp * 0x1p-96f * (qnorm + Rb + ex + 1.0f);
    if (M == LIRA_METRIC_L2) {
        const float s = qnorm + Rb;
        return (2.0f * ed + (1.05f * 8.0f + 2.01f + 2.0f) * 0x1p-24f * s * s) * (1.0f + 0x1p-18f) + 0x1p-125f;
    }
    const float aq = __builtin_fabsf(qc);
    return (ed + (1.01f * qnorm * Rb + 2.02f * aq + qnorm * (Rb + ex) + (dd + 2.0f) * qnorm * Rx) * 0x1p-24f) * 1.05f +
           0x1p-125f;
}

// the screened score of a candidate from wv = fl(dot - xadj), per row qv = qn (L2)
// or qc (IP): L2 s~ = fl(qn - 2 wv) (k_screen_m: fma(-2, dot, fl(qn + 2 xadj));
// this form's extra rounding is in errE_r's 2 u s^2); IP s~ = -fl(wv + qc)
template <int M>
__device__ __forceinline__ u64 rkey(float wv, float qv, uint32_t pos) {
    const float s = M == LIRA_METRIC_L2 ? qv - 2.0f * wv : -(wv + qv);
    return ((u64)f2ord(s) << 32) | pos;
}

// Buffered survivors carry fl(dot - xadj) instead of the score: a wkey is
// (f2ord(-wv), storage position), ascending in the score for a fixed row (both
// metrics); the buffers hold its high word and the position in the item (u16),
// and it is converted to the list key (rkey, the same arithmetic) when merged,
// where the row's qn / qc is one broadcast read (the selection needs no LDS read)
template <int M>
__device__ __forceinline__ u64 wkey_to_key(u64 wk, float qv) {
    return rkey<M>(-ord2f((uint32_t)(wk >> 32)), qv, (uint32_t)wk);
}

// the bound on the final k-th exact score from a list's k-th screened key (bound_P)
__device__ __forceinline__ float bound_of(u64 kk, float er, float gP) {
    return kk != kEmptyKey ? rup(rup(key_score(kk) + er) * gP) + 0x1p-125f : __builtin_inff();
}
// s_lim's T part: L2 (T + d 2^-140) / (1 - g), IP T (the error is all in E)
template <int M>
__device__ __forceinline__ float lim_of(float T, float invF) {
    if (!(T < 3e38f)) return __builtin_inff();
    return M == LIRA_METRIC_L2 ? rup(rup(fmaxf(T, 0.0f) + 0x1p-125f) * invF) : T;
}

// key e (runtime, < 32 RL) of a half-wave list, broadcast to the lane's half
// (masks, not a select chain: hipcc turned the chain into a scratch array indexed
// by e >> 5)
template <int RL>
__device__ __forceinline__ u64 list_at(const u64 (&lst)[RL], int e) {
    const int r = __builtin_amdgcn_readfirstlane(e >> 5);
    u64 x = 0;
#pragma unroll
    for (int i = 0; i < RL; ++i) x |= lst[i] & (0ull - (u64)(r == i));
    return shfl64(x, (lane_id() & 32) + (e & 31));
}

// A row list's merge with the keys it evicts (spill lists on): per half, lst <- the
// 32 RL smallest of lst U batch, and ev = the 32 largest (what half_merge_batch1 drops:
// the list's first 32 (RL - 1) keys are below its last 32)
template <int RL>
__device__ __forceinline__ u64 merge_evict(u64 (&lst)[RL], u64 batch) {
    u64 b[1] = {batch};
    half_sort<1>(b);
    const u64 rev = rev32_u64(b[0]);
    const u64 ev = kmax(lst[RL - 1], rev);
    lst[RL - 1] = kmin(lst[RL - 1], rev);
    half_bitonic_merge<RL>(lst);
    return ev;
}

// Keys a row list evicted that the merge may still need go to the query's spill
// list (k_smerge rechecks them like list keys, so a full list needs no re-scan):
// the ones within lim(T) + E for the row's current T -- its list's new k-th bound
// or the T its thresholds use, both >= the final one -- by the screen's own
// rounding, which is above k_smerge's s_lim(T, E) (lira_bounds.hpp).  Per half-wave
// (hv: this lane's half holds the row).  Past scap records the query's count shows
// the overflow and k_smerge re-scans its full lists instead.
template <int M>
__device__ __forceinline__ void spill_evicted(const RArgs &a, u64 ev, bool hv, u64 kth, float er, float Tc, int pr) {
    const float T = fminf(bound_of(kth, er, a.gP), Tc);
    const float lim = rup(lim_of<M>(T, a.invF) + er);
    const bool sp = hv && pr >= 0 && ev != kEmptyKey && key_score(ev) <= lim;
    const u64 m = __ballot(sp);
    if (!m) return;
    // (one atomic per half-wave: the halves may hold different queries' rows)
    const int lane = lane_id();
    const u64 hm = m & (lane < 32 ? 0xffffffffull : 0xffffffff00000000ull);
    const int hl0 = lane & 32;
    unsigned base = 0;
    const int q = pr / a.nprobe;
    if ((lane & 31) == 0 && hm) base = atomicAdd(a.scnt + q, (unsigned)__popcll(hm));
    base = (unsigned)__shfl((int)base, hl0, 64);
    const unsigned at = base + (unsigned)__popcll(hm & ((1ull << lane) - 1ull));
    if (sp && at < (unsigned)a.scap)
        a.spill[(int64_t)q * a.scap + at] = make_uint4((uint32_t)ev, (uint32_t)(ev >> 32), __float_as_uint(er), 0u);
}

// Merge this wave's buffers of two rows (half-wave h: row rows[h], BC keys; a
// second row < 0: half 1 idles) into their shared lists, under the rows' LDS
// locks (taken in row order, row0 < row1: no two waves wait on each other):
// raise each row's running error bound to the wave's first (readers take the
// list's k-th key, then the bound: program order in both), half-wave merges,
// publish the query's bound where a list's k-th improved.  One row per half: a
// single-row merge left half of the wave idle in every flush.
template <int M, int RL, int BC, int BCS = BC | 1>
__device__ __forceinline__ void flush_rows(u64 *lists, u64 *kth_s, const uint32_t *mbh, const uint16_t *mbl,
                                           uint32_t pos_base, int *lock_s, uint32_t *erun_s, uint32_t *opub_s,
                                           const int *pair_s, int row0, int row1, int ew0, int ew1, int k,
                                           const float4 *rec_s, const RArgs &a, float Tc0, float Tc1) {
    constexpr int K2 = 32 * RL;
    const int lane = opaque(lane_id()), hl = lane & 31;  // (opaque: addresses computed here, not hoisted)
    const bool h1 = lane >= 32, act = !h1 || row1 >= 0;
    const int row = h1 && row1 >= 0 ? row1 : row0;
    if (lane == 0) {
        while (atomicCAS(lock_s + row0, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
        atomicMax(erun_s + row0, (uint32_t)ew0);
    }
    if (lane == 32 && row1 >= 0) {
        while (atomicCAS(lock_s + row1, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
        atomicMax(erun_s + row1, (uint32_t)ew1);
    }
    asm volatile("" ::: "memory");
    u64 lst[RL];
#pragma unroll
    for (int r = 0; r < RL; ++r) lst[r] = lists[row * K2 + r * 32 + hl];
    const u64 b = act && hl < BC ? wkey_to_key<M>(((u64)mbh[row * BCS + hl] << 32) | (pos_base + mbl[row * BCS + hl]),
                                       rec_s[row].x)
                      : kEmptyKey;
    u64 ev = kEmptyKey;
    if (a.spill)
        ev = merge_evict<RL>(lst, b);
    else
        half_merge_batch1<RL>(lst, b);
    if (act) {
#pragma unroll
        for (int r = 0; r < RL; ++r) lists[row * K2 + r * 32 + hl] = lst[r];
    }
    const u64 kk = list_at<RL>(lst, k - 1);  // (per half)
    if (hl == 0 && act) {
        kth_s[row] = kk;
        if (kk != kEmptyKey && a.qbound) {
            const int pr = pair_s[row];
            if (pr >= 0) {
                const uint32_t P = f2ord(bound_of(kk, __uint_as_float(erun_s[row]), a.gP));
                if (P < opub_s[row]) {
                    opub_s[row] = P;
                    atomicMin(a.qbound + pr / a.nprobe, P);
                }
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (LDS in order: the lists are written before the unlocks)
    if (hl == 0 && act) *(volatile int *)(lock_s + row) = 0;
    __builtin_amdgcn_wave_barrier();
    if (a.spill)  // (after the unlocks: the atomics' round trips hold no other wave)
        spill_evicted<M>(a, ev, act, kk, __uint_as_float(erun_s[row]), h1 ? Tc1 : Tc0, pair_s[row]);
}

// Merge this wave's full row buffers into the lists, then move the survivor
// queue into the buffers (LDS atomic slots), merging every buffer that fills,
// until the queue is empty.
template <int M, int RL, int BC, int BCS = BC | 1>
__device__ __forceinline__ void drain_buffers(u64 *lists, u64 *kth_s, uint32_t *mbh, uint16_t *mbl, int *mybufc, int *lock_s,
                                              uint32_t *erun_s, uint32_t *opub_s, const int *pair_s,
                                              const float4 *rec_s, const u64 *oq_key, uint32_t pos_base, int nq,
                                              float Ew, int k, const RArgs &a, float Tc) {
    const int lane = opaque(lane_id());
    auto flush_full = [&]() {
        u64 full = __ballot(mybufc[lane] >= BC);  // lane = row
        while (full) {
            const int row0 = __builtin_ctzll(full);
            full &= full - 1;
            const int row1 = full ? __builtin_ctzll(full) : -1;
            if (full) full &= full - 1;
            const int r1 = row1 >= 0 ? row1 : row0;
            flush_rows<M, RL, BC>(lists, kth_s, mbh, mbl, pos_base, lock_s, erun_s, opub_s, pair_s, row0, row1,
                                  __builtin_amdgcn_readlane(__float_as_int(Ew), row0),
                                  __builtin_amdgcn_readlane(__float_as_int(Ew), r1), k, rec_s, a,
                                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Tc), row0)),
                                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Tc), r1)));
            if (lane == 0) mybufc[row0] = 0;
            if (lane == 0 && row1 >= 0) mybufc[row1] = 0;
            __builtin_amdgcn_wave_barrier();
        }
    };
    flush_full();
    for (int e0 = 0; e0 < nq; e0 += 64) {
        const int e = e0 + lane;
        bool pend = e < nq;
        // (queue entry: fl(-xadj + dot) bits | row << 16 | the candidate's position in
        // the item; the selection does no conversion)
        const u64 q = pend ? oq_key[e] : 0ull;
        const int row = (int)((q >> 16) & 63u);
        const uint32_t kh = pend ? f2ord(-__uint_as_float((uint32_t)(q >> 32))) : 0u;  // (wkey's high word)
        while (__any(pend)) {
            if (pend) {
                const int slot = atomicAdd(mybufc + row, 1);
                if (slot < BC) {
                    mbh[row * BCS + slot] = kh;
                    mbl[row * BCS + slot] = (uint16_t)(q & 0xffffu);
                    pend = false;
                }
            }
            __builtin_amdgcn_wave_barrier();
            // rows the round filled (a lane that overflowed left its row's count above BC)
            if (mybufc[lane] > BC) mybufc[lane] = BC;
            __builtin_amdgcn_wave_barrier();
            flush_full();
        }
    }
}

template <int NC, int M, int RL, int W>  // NC: 32-dim chunks (dpad = 32 NC); M: metric; RL: list registers; W: waves
__global__ __launch_bounds__(64 * W, W == 8 ? 1 : 2) void k_screen_r(RArgs a) {
    typedef RSmem<RL, W> S;
    constexpr int QR = S::QR, K2 = S::K2, NRG = S::NRG, BC = S::BC, NT = 64 * W;
    constexpr int NSTEP = 8 * NRG;  // selection steps per tile: (row group, register, candidate pair)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    u64 *lists = (u64 *)(smem + S::lists);
    uint32_t *bufs = (uint32_t *)(smem + S::bufs);
    uint16_t *bufl = (uint16_t *)(smem + S::bufl);
    int *bufc = (int *)(smem + S::bufc);
    float *hs = (float *)(smem + S::hs);
    float2 *tst = (float2 *)(smem + S::tst);
    float *trs = (float *)(smem + S::trs);
    int *pair_s = (int *)(smem + S::pair);
    float4 *rec_s = (float4 *)(smem + S::qn);
    const uint4 *aq_s = (const uint4 *)(smem + S::aq);
    uint32_t *erun_s = (uint32_t *)(smem + S::erun);
    int *lock_s = (int *)(smem + S::lock);
    uint32_t *opub_s = (uint32_t *)(smem + S::opub);
    int *meta = (int *)(smem + S::meta);
    u64 *kth_s = (u64 *)(smem + S::kth);
    __shared__ int xq[9];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, cj = lane & 15;
    const int k = a.k;
    const float dp = (float)a.dpad, dd = (float)a.d;
    uint32_t *mybuf = bufs + wave * S::WS;
    uint16_t *mybufl = bufl + wave * S::WS;
    int *mybufc = bufc + wave * 64;
    float *myh = hs + wave * 64;
    u64 *oq_key = (u64 *)(smem + S::oqk) + wave * kROCap;
    const bool TRI = a.tstat != nullptr;
    // B fragment: the lane's byte offset inside a tile's 32-dim chunk
    const uint32_t lane_off = (uint32_t)((g >> 1) * 4096 + (g & 1) * 1024 + cj * 16);
    const int64_t tile_bytes = a.dpad * 64 * 4;
    unsigned long long n_tiles = 0, n_skip = 0, n_surv = 0;

    const int bpc_near_d = __builtin_amdgcn_readfirstlane(a.head[19]);
    // Items are claimed by the last wave's lane 0 (its tiles are u = 3, 7, ...: the
    // fewest when the item's tile count is not a multiple of 4), right after its
    // tile loop: the claim's atomic and the entry's load overlap the other waves'
    // last tiles instead of holding every wave at the item's first barrier
    int qx = 0, qtries = 0;
    auto claim_into_meta = [&]() {
        const int it = claim_item(a.head, xq, qx, qtries);
        const int4 e = it >= 0 ? a.itab[it] : make_int4(0, 0, 0, 0);
        meta[0] = it >= 0;
        meta[1] = e.x;
        meta[2] = e.y;
        meta[3] = e.z;
        meta[6] = e.w;  // (the query block's index over all buckets)
        meta[4] = 0;  // the item's max tile radius / hi residual (bits), max-reduced in its prologue
        meta[5] = 0;
    };
    if (tid < 9) xq[tid] = a.head[10 + tid];
    __syncthreads();
    if (wave == W - 1 && lane == 0) {
        qx = xcd_id();
        claim_into_meta();
    }
    __syncthreads();
    for (;;) {
        if (!meta[0]) break;
        const int vp = __builtin_amdgcn_readfirstlane(meta[1]);
        const int qb = __builtin_amdgcn_readfirstlane(meta[2]);
        const int ch = __builtin_amdgcn_readfirstlane(meta[3]);
        const int p = vp >= a.n_lists ? vp - a.n_lists : vp;
        const int tile0 = __builtin_amdgcn_readfirstlane(a.tile_off[p]);
        const int ntl = __builtin_amdgcn_readfirstlane(a.tile_off[p + 1]) - tile0;
        // chunk ch of the bucket: group 0 (each query's nearest partition) has a
        // first chunk of head[21] blocks, then chunks of head[19]; the others a.bpc
        const bool g0 = vp < a.n_lists && a.n_virt > a.n_lists;
        const int b0 = __builtin_amdgcn_readfirstlane(a.head[21]);
        const int blk0 = g0 ? (ch == 0 ? 0 : b0 + (ch - 1) * bpc_near_d) : ch * a.bpc;
        const int nbk = g0 ? (ch == 0 ? b0 : bpc_near_d) : a.bpc;
        const int tb_begin = blk0 * 4;
        const int nt = min(ntl, tb_begin + nbk * 4) - tb_begin;  // the item's tiles (<= kRMaxTiles)
        const int qblk = __builtin_amdgcn_readfirstlane(meta[6]);
        const int tbase = tile0 + tb_begin;
        const float R = a.rmax[p];
        const float Rx = M == LIRA_METRIC_IP ? a.rmaxx[p] : 0.0f;
        int u = wave;
        // B operands: a ring of NC chunks of [candidate group] -- the whole next
        // tile: chunk c's slot is reloaded with the next tile's chunk c as soon as its
        // MFMAs have issued, so a tile's loads have a whole tile (MFMAs + selection)
        // to land (two chunks ahead, round 4's ring at d = 128, left chunks 2-3 of
        // every tile waiting on HBM).  The wave's first tile is requested before the
        // prologue (under its loads and barriers), and again only if skipped.
        // (NC = 0: dpad > 128, the dims streamed two chunks ahead -- a whole tile is
        // dpad / 2 bytes per lane -- and the A operands too, see SA below)
        constexpr int RS = NC == 0 ? 2 : NC;
        rbf16x8 B[RS][4];
        rf4 xa_n = (rf4)(0.0f);  // the next tile's xadj (candidates 4 cj .. + 3)
        // (xadj first, then B: the loop's first use is xa, so on every path into
        // the tile loop the compiler's wait for it leaves the B loads in flight)
        auto load_first = [&]() {
            const char *base = a.Xb + (int64_t)(tbase + u) * tile_bytes + lane_off;
            xa_n = *(const rf4 *)(a.xadj + (int64_t)(tbase + u) * 64 + 4 * cj);
#pragma unroll
            for (int c = 0; c < RS; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i) B[c][i] = *(const rbf16x8 *)(base + c * 8192 + i * 256);
        };
        if (u < nt) load_first();

        // ---- item prologue: row records, lists, tile statistics
        const int nval = a.cnt[vp] - qb * QR;
        const int my_pair = lane < QR && lane < nval ? a.qlist[a.qoff[vp] + qb * QR + lane] : -1;  // lane = row
        const float4 qrec = my_pair >= 0 ? a.QN[my_pair] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float my_qres = my_pair >= 0 ? a.QE[my_pair] : 0.0f;
        const int my_q = my_pair >= 0 ? my_pair / a.nprobe : -1;
        // a later chunk of a nearest partition waits for the query block's first
        // chunk, whose epilogue publishes the rows' bounds (queued ahead of it in
        // the same queue, so it is claimed and running: no wait can deadlock).  The
        // bounds are hints -- a stale or missing one is only looser -- so the wait
        // is also bounded (~2^14 polls).  Polls and the flag are atomics: they act
        // at the memory side, past the XCDs' non-coherent L2s.
        if (g0 && ch > 0 && a.done0 && tid == 0)
            for (int it = 0; it < (1 << 14) && atomicAdd(a.done0 + qblk, 0) == 0; ++it) __builtin_amdgcn_s_sleep(8);
        __syncthreads();  // (the previous item's epilogue is done with the LDS state)
        if (wave == 0) {
            pair_s[lane] = my_pair;
            rec_s[lane] = make_float4(qrec.x, qrec.y, my_qres, qrec.w);
            erun_s[lane] = 0u;
            lock_s[lane] = 0;
            opub_s[lane] = ~0u;
            kth_s[lane] = kEmptyKey;
        }
        mybufc[lane] = 0;
        {
            uint4 *l4 = (uint4 *)lists;
            const uint4 e4 = make_uint4(~0u, ~0u, ~0u, ~0u);
            for (int i = tid; i < QR * K2 / 2; i += NT) l4[i] = e4;
        }
        if (TRI) {
            float rb = 0.0f, hr = 0.0f;
            for (int i = tid; i < nt; i += NT) {
                const float2 t2 = a.tstat[tbase + i];
                tst[i] = t2;
                rb = fmaxf(rb, t2.y);
                if (a.tres) {
                    const float tr = a.tres[tbase + i];
                    trs[i] = tr;
                    hr = fmaxf(hr, tr);
                }
            }
            atomicMax((uint32_t *)meta + 4, __float_as_uint(rb));  // (>= 0: ordered as integers)
            if (a.tres) atomicMax((uint32_t *)meta + 5, __float_as_uint(hr));
        }
        __syncthreads();

        // A operands into LDS, in fragment order: [chunk c][row group rg][lane (g, j)]
        // = row 16 rg + j, dims 32 c + 8 g .. + 7 (each wave reads 1 KiB per (c, rg))
        // (SA: none -- they are read from the per-pair records as the tiles stream)
        for (int e = tid; e < NC * NRG * 64; e += NT) {
            const int l = e & 63, rg = (e >> 6) % NRG, c = e / (64 * NRG);
            const int pr = pair_s[16 * rg + (l & 15)];
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (pr >= 0) v = *(const uint4 *)(a.QH + (int64_t)pr * a.dpad + 32 * c + 8 * (l >> 4));
            ((uint4 *)(smem + S::aq))[e] = v;
        }
        __syncthreads();
        // SA (NC = 0, dpad > 128: GIST1M's 960 dims would need 120 KB of LDS for the
        // rows' hi parts): each wave reads the A fragments of chunk c from QH, the rows'
        // records (L2-resident: one item's rows are 64 x dpad x 2 bytes), in a ring two
        // chunks ahead like the B fragments.  A padding row reads row 0's record: its
        // products are garbage in a row that never passes.
        constexpr bool SA = NC == 0;
        const int nca = SA ? (int)(a.dpad >> 5) : NC;
        uint32_t arow[NRG];  // (element offsets into QH: 32-bit, on the uniform base)
        rbf16x8 Ar[2][NRG];
        if (SA) {
#pragma unroll
            for (int rg = 0; rg < NRG; ++rg) {
                const int pr = pair_s[16 * rg + (lane & 15)];
                arow[rg] = (uint32_t)((pr >= 0 ? pr : pair_s[0]) * (int)a.dpad + 8 * (lane >> 4));
#pragma unroll
                for (int h = 0; h < 2; ++h) Ar[h][rg] = *(const rbf16x8 *)(a.QH + arow[rg] + 32 * h);
            }
        }

        // ---- per-row bound state (lane = row; qbound is always set here)
        // my_qv: L2 qn = fl(||q'||^2), IP qc = fl(q.c); my_dq: L2 fl(||q - c||)
        const float my_qv = qrec.x, my_qnorm = qrec.y, my_dq = qrec.w;
        const uint32_t *pub_at = a.qbound + (my_q >= 0 ? my_q : 0);  // (a padding row reads query 0's: unused)
        uint32_t pub = __hip_atomic_load(pub_at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        float Tc = -1.0f, triA = -__builtin_inff(), triB = __builtin_inff();
        // The screening error bound is the item's (its largest tile radius and hi
        // residual: err_E is monotone in both), so a row's threshold changes only
        // when its T does; Ew = the bound of every key this item lists (lane = row)
        const float Rb_item = TRI ? fminf(R, rup(__uint_as_float((uint32_t)meta[4]))) : R;
        const float hres_item = TRI && a.tres ? __uint_as_float((uint32_t)meta[5]) : -1.0f;
        const float Ew = my_pair >= 0 ? errE_r<M>(my_qnorm, Rb_item, hres_item, my_qres, dp, my_qv, Rx, dd) : 0.0f;
        // (IP) the Cauchy-Schwarz skip's slack: qc's rounding, search.cpp's exact sum
        const float slk = M == LIRA_METRIC_IP && my_pair >= 0
            ? (1.01f * __builtin_fabsf(my_qv) + (dd + 2.0f) * my_qnorm * Rx) * 0x1p-24f * 1.02f + 0x1p-120f : 0.0f;
        const int g4 = opaque(4 * g);  // (selection rows: 16 rg + g4 + reg)
        // T: the row's bound on its final k-th exact score (shared list, published bound).
        // No divergent branch (the published bound's load stays countable for the
        // compiler's waits: a conditional one cost a vmcnt(0) per tile).  The next
        // published bound is requested only inside the tile loop (refresh), ahead of
        // the tile's other loads: on every path into the loop the outstanding loads
        // are then the pub load followed by the tile's, and its wait leaves them in flight
        auto update_T = [&](bool refresh) {
            const u64 kk = kth_s[lane];
            asm volatile("" ::: "memory");  // (the list's key first, then its bound: see flush_row)
            const float er = __uint_as_float(erun_s[lane]);
            float T = bound_of(kk, er, a.gP);
            T = fminf(T, ord2f(pub));  // (~0u, nothing published: a NaN, which fminf ignores)
            if (refresh) pub = __hip_atomic_load(pub_at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__any(T != Tc)) {  // (recomputed for every lane: an unchanged T gives the same values)
                Tc = T;
                const bool fin = T < 3e38f;
                const float Ac = lim_of<M>(T, a.invF);
                if (M == LIRA_METRIC_L2) {
                    // (v_sqrt_f32, <= 1 ulp: inside rup's 2^-20 margin)
                    const float rad = rup(__builtin_amdgcn_sqrtf(Ac));
                    triA = my_pair < 0 ? __builtin_inff() : fin ? rdn(rdn(my_dq) - rad) : -__builtin_inff();
                    triB = my_pair < 0 ? -__builtin_inff() : fin ? rup(rup(my_dq) + rad) : __builtin_inff();
                } else {
                    // a tile can hold a candidate of exact score <= T only if its largest
                    // radius reaches (-qc - slack - T) / ||q|| (||q|| rounded up)
                    triA = my_pair < 0 ? __builtin_inff()
                           : fin && my_qnorm > 0.0f ? rdn(rdn(rdn(-my_qv - slk) - Ac) / my_qnorm) : -__builtin_inff();
                    triB = my_pair < 0 ? -__builtin_inff() : __builtin_inff();
                }
                // pass iff fl(-xadj + dot) >= h (lane = row), then the rows in selection order
                float h = __builtin_inff();
                if (my_pair >= 0) {
                    h = -__builtin_inff();
                    if (fin) {
                        const float lim = rup(Ac + Ew);
                        if (M == LIRA_METRIC_L2) {
                            const float sq = my_qnorm + Rb_item;
                            h = rdn(0.5f * (my_qv - lim) - (__builtin_fabsf(my_qv) + __builtin_fabsf(lim)) * 0x1p-22f -
                                    1.06f * 0x1p-24f * sq * sq);
                        } else {  // s~ = -fl(wv + qc) <= lim  =>  wv >= -lim - qc - (|lim| + |qc|) 2^-22
                            h = rdn(rdn(-lim - my_qv) - (__builtin_fabsf(my_qv) + __builtin_fabsf(lim)) * 0x1p-22f);
                        }
                    }
                    h = fmaxf(h, -3.40282347e38f);  // (padding, xadj = +inf, never passes)
                }
                myh[lane] = h;
                __builtin_amdgcn_wave_barrier();
            }
        };
        // tile u is needed by no row (wave-uniform)
        auto skip = [&](int u) {
            if (!TRI) return false;
            const float2 r = tst[u];
            return __all(r.y < triA || r.x > triB) != 0;
        };

        update_T(false);
        if (u < nt && skip(u)) {
            do {
                ++n_skip;
                u += W;
            } while (u < nt && skip(u));
            if (u < nt) load_first();
        }
        int ovf = 0;  // survivor queue fill (wave-uniform)
        // survivor queue -> this wave's row buffers (full ones merged into the lists)
        auto drain = [&]() {
            drain_buffers<M, RL, BC>(lists, kth_s, mybuf, mybufl, mybufc, lock_s, erun_s, opub_s, pair_s, rec_s, oq_key,
                                 (uint32_t)tbase * 64u, ovf, Ew, k, a, Tc);
            ovf = 0;
        };

        while (u < nt) {
            const rf4 xa = xa_n;
            // ---- the row bounds (thresholds rewritten where one changed)
            update_T(true);

            // ---- the next tile of this wave (skip test with the current intervals)
            int un = u + W;
            while (un < nt && skip(un)) {
                ++n_skip;
                un += W;
            }
            const int ul = un < nt ? un : u;  // (the last tile's loads repeat the current tile)
            const char *cbase = a.Xb + (int64_t)(tbase + u) * tile_bytes + lane_off;
            const char *nbase = a.Xb + (int64_t)(tbase + ul) * tile_bytes + lane_off;
            xa_n = *(const rf4 *)(a.xadj + (int64_t)(tbase + ul) * 64 + 4 * cj);
            // the rows' thresholds in selection order (read under the MFMAs)
            rf4 hv[NRG];
#pragma unroll
            for (int rg = 0; rg < NRG; ++rg) hv[rg] = *(const rf4 *)(myh + 16 * rg + g4);

            // ---- QR rows x 64 candidates: acc = -xadj + dot (the first chunk's MFMAs
            // take C = -xadj of their candidate; lane (g, j) holds candidates 4 j + i
            // of rows 4 g + reg, so C is the same for every row group); each B
            // fragment's slot reloaded after its NRG MFMAs
            rf4 acc[NRG][4];
            // SA: chunk pairs (slots 0, 1), the first pair peeled (C = -xadj there)
            auto sa_chunk = [&](int c, int h, bool first) {
                const int cn = c + 2;
                rbf16x8 Acur[NRG];
#pragma unroll
                for (int rg = 0; rg < NRG; ++rg) Acur[rg] = Ar[h][rg];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const rf4 cx = (rf4)(-xa[i]);
#pragma unroll
                    for (int rg = 0; rg < NRG; ++rg)
                        acc[rg][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Acur[rg], B[h][i], first ? cx : acc[rg][i],
                                                                             0, 0, 0);
                    B[h][i] = cn < nca ? *(const rbf16x8 *)(cbase + (int64_t)cn * 8192 + i * 256)
                                       : *(const rbf16x8 *)(nbase + (int64_t)(cn - nca) * 8192 + i * 256);
                }
                const int ca = cn < nca ? cn : cn - nca;  // (the A ring runs on into the next tile: the same rows)
#pragma unroll
                for (int rg = 0; rg < NRG; ++rg) Ar[h][rg] = *(const rbf16x8 *)(a.QH + arow[rg] + 32 * ca);
                __builtin_amdgcn_sched_barrier(0);
            };
            if (SA) {
                sa_chunk(0, 0, true);
                sa_chunk(1, 1, false);
#pragma unroll 1
                for (int c0 = 2; c0 < nca; c0 += 2) {
                    sa_chunk(c0, 0, false);
                    sa_chunk(c0 + 1, 1, false);
                }
            }
            // per chunk: the A fragments (LDS), this chunk's MFMAs, the slot's
            // reloads; a scheduling barrier per chunk keeps the reloads where they are
            // (left alone, hipcc sank them next to their consumers)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int sl = c % RS, cn = c + RS;  // slot; the chunk that goes into it next
                rbf16x8 Acur[NRG];
#pragma unroll
                for (int rg = 0; rg < NRG; ++rg) Acur[rg] = __builtin_bit_cast(rbf16x8, aq_s[(c * NRG + rg) * 64 + lane]);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const rf4 cx = (rf4)(-xa[i]);
#pragma unroll
                    for (int rg = 0; rg < NRG; ++rg)
                        acc[rg][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Acur[rg], B[sl][i], c == 0 ? cx : acc[rg][i],
                                                                             0, 0, 0);
                    B[sl][i] = cn < NC ? *(const rbf16x8 *)(cbase + cn * 8192 + i * 256)
                                       : *(const rbf16x8 *)(nbase + (cn - NC) * 8192 + i * 256);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            ++n_tiles;

            // ---- selection: pass iff acc = -xadj + dot >= h.  Per (row group, register)
            // entry e = 4 rg + reg, lane group g holds row 16 rg + 4 g + reg: four
            // compares into wave masks (one per candidate slot i), skipped together
            // when all are empty; each non-empty mask's lanes append (wv, position,
            // row) to the wave's survivor queue at slots from the mask's prefix count.
            // The pass runs over (entry, half) steps h = 2 e + (i >> 1); a step that
            // would overflow the queue stops it there, the queue is drained (one
            // inlined call site) and the pass resumes at that step (rare)
            // (MXPRE, 32-row variants: each entry first compares the max of its four
            // slots -- one ballot instead of four on the sparse latent tiles; measured
            // slower on the 64-row SIFT1M mixture, so not there)
            constexpr bool MXPRE = RL >= 2;
            const uint32_t lpos0 = (uint32_t)(u * 64 + 4 * cj);
            for (int s0 = 0;;) {
                // (the accumulators as if redefined: keeps the compares from being
                // hoisted out of this loop, which cost 64 masks held in SGPRs)
#pragma unroll
                for (int rg = 0; rg < NRG; ++rg)
#pragma unroll
                    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(acc[rg][i]));
                // (likewise the entries' low words: row << 16 | position, from one value
                // per pass -- hoisted, the 32 precomputed words were spilled)
                const uint32_t low0 = (uint32_t)opaque((int)(((uint32_t)g4 << 16) | lpos0));
                int stop = NSTEP;
#pragma unroll
                for (int rg = 0; rg < NRG; ++rg) {
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) {
                        const int e = 4 * rg + reg;
                        if (2 * e + 1 < s0 || 2 * e >= stop) continue;
                        const float hp = hv[rg][reg];
                        if (MXPRE) {  // (NaN-ignoring max: a NaN slot fails its own compare either way)
                            const float mx = fmaxf(fmaxf(acc[rg][0][reg], acc[rg][1][reg]),
                                                   fmaxf(acc[rg][2][reg], acc[rg][3][reg]));
                            if (!__ballot(mx >= hp)) continue;
                        }
                        u64 m[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) m[i] = __ballot(acc[rg][i][reg] >= hp);
                        if (!(m[0] | m[1] | m[2] | m[3])) continue;
                        const uint32_t low = low0 + ((uint32_t)(16 * rg + reg) << 16);
#pragma unroll
                        for (int hf = 0; hf < 2; ++hf) {
                            const int h = 2 * e + hf;
                            if (h < s0 || h >= stop) continue;
                            const u64 ma = m[2 * hf], mb = m[2 * hf + 1];
                            const int na = popc64(ma), n = na + popc64(mb);
                            if (!n) continue;
                            if (ovf + n > kROCap) {  // (n <= 128: fits once drained)
                                stop = h;
                                continue;
                            }
                            n_surv += (unsigned long long)n;
                            // queue entry: fl(-xadj + dot) bits | row << 16 | position in the item
                            if ((ma >> lane) & 1ull)
                                oq_key[ovf + mbcnt64(ma)] = ((u64)__float_as_uint(acc[rg][2 * hf][reg]) << 32) | (low + 2u * hf);
                            if ((mb >> lane) & 1ull)
                                oq_key[ovf + na + mbcnt64(mb)] =
                                    ((u64)__float_as_uint(acc[rg][2 * hf + 1][reg]) << 32) | (low + 2u * hf + 1u);
                            ovf += n;
                        }
                    }
                }
                if (stop == NSTEP) break;
                drain();
                s0 = stop;
            }
            u = un;
        }
        if (ovf) drain();
        if (wave == W - 1 && lane == 0) claim_into_meta();  // (the next item; read after the barriers below)

        // ---- item epilogue: every wave's buffers into the lists (rows split over
        // the waves, two per pass: one per half-wave), then the lists out
        if (mybufc[lane] > 0) atomicMax(erun_s + lane, __float_as_uint(Ew));
        __syncthreads();
        const int ln = opaque(lane);  // (lane-derived addresses computed here, not hoisted)
        constexpr int RPW = QR / W;  // rows per wave
#pragma unroll 1
        for (int j = 0; j < RPW; j += 2) {
            const int hl = ln & 31, row = wave * RPW + j + (ln >> 5);
            int n = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) n += bufc[w * 64 + row];
            if (!__any(n > 0)) continue;
            const float qv_r = rec_s[row].x;
            for (int r0 = 0; __any(n > r0); r0 += 32) {
                const int e = r0 + hl;
                u64 b = kEmptyKey;
                if (e < n) {
                    int w = 0, off = e;  // (the wave buffer holding key e of the row's concatenation)
                    while (off >= bufc[w * 64 + row]) off -= bufc[w++ * 64 + row];
                    const int e2 = w * S::WS + row * S::BCS + off;
                    b = wkey_to_key<M>(((u64)bufs[e2] << 32) | ((uint32_t)tbase * 64u + bufl[e2]), qv_r);
                }
                u64 lst[RL];
#pragma unroll
                for (int r = 0; r < RL; ++r) lst[r] = lists[row * K2 + r * 32 + hl];
                if (a.spill) {
                    const u64 ev = merge_evict<RL>(lst, b);
#pragma unroll
                    for (int r = 0; r < RL; ++r) lists[row * K2 + r * 32 + hl] = lst[r];
                    spill_evicted<M>(a, ev, true, list_at<RL>(lst, k - 1), __uint_as_float(erun_s[row]),
                                     __shfl(Tc, row, 64), pair_s[row]);
                } else {
                    half_merge_batch1<RL>(lst, b);
#pragma unroll
                    for (int r = 0; r < RL; ++r) lists[row * K2 + r * 32 + hl] = lst[r];
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        // (sorted lists: the keys, the first empty one and the last slot are all
        // k_smerge reads -- its walk stops at the first key beyond its limit)
#pragma unroll 1
        for (int j = 0; j < RPW; j += 2) {
            const int hl = ln & 31, row = wave * RPW + j + (ln >> 5);
            const int pr = pair_s[row];
            u64 key[RL];
            int nv = 0;
#pragma unroll
            for (int r = 0; r < RL; ++r) {
                key[r] = lists[row * K2 + r * 32 + hl];
                const u64 full = __ballot(key[r] != kEmptyKey);
                nv += __builtin_popcount((uint32_t)(ln >> 5 ? full >> 32 : full));
            }
            if (pr >= 0) {
                u64 *dst = a.partial + ((int64_t)pr * a.nch_max + ch) * K2;
#pragma unroll
                for (int r = 0; r < RL; ++r) {
                    const int e = r * 32 + hl;
                    if (e <= nv || e == K2 - 1) dst[e] = key[r];
                }
            }
        }
        if (my_pair >= 0) {
            const float er = __uint_as_float(erun_s[lane]);
            a.pE[(int64_t)my_pair * a.nch_max + ch] = fmaxf(er, 0x1p-126f);  // (>= every listed key's bound)
            const u64 kk = lists[lane * K2 + k - 1];
            if (a.qbound && kk != kEmptyKey) atomicMin(a.qbound + my_q, f2ord(bound_of(kk, er, a.gP)));
        }
        if (g0 && ch == 0 && a.done0) {  // the query block's later chunks may start
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's published bounds landed)
            __syncthreads();
            if (tid == 0) atomicAdd(a.done0 + qblk, 1);
        }
    }
    if (a.stats && lane == 0) {
        atomicAdd(a.stats + 0, n_tiles * (unsigned long long)QR * 64ull);  // (row, candidate) pairs screened
        atomicAdd(a.stats + 2, n_tiles);                                   // tiles computed (of 64 candidates)
        atomicAdd(a.stats + 4, n_skip);                                    // tiles skipped by the triangle test
        atomicAdd(a.stats + 7, n_surv);                                    // survivors appended
    }
}

// ---- k_seed_r: the screened seed bound + per-pair records --------------------
// One wave per query.  The query's slot-0 record first (no filter: its own list),
// then the bound: the first NT tiles of that list screened on the matrix cores
// exactly as k_screen_r screens them (A = the query row's hi parts in row 0 of the
// 16 x 32 operand, the other 15 rows zero: 2 NT NC MFMAs per query, ~16x the useful
// MACs, still far below the 2 NT x 64 x d sequential fp32 sums of k_seed_t), every
// screened score within errE_r of search.cpp's exact one, so the k-th smallest of the
// 64 NT keys + E bounds the query's final k-th exact score (bound_P: k distinct
// candidates of one list).  Then the records of slots 1.. under that bound (the
// partition filter), as k_seed_t<..., PAIRS> / k_pairs.
template <int NC, int M, int NT>
__global__ __launch_bounds__(256) void k_seed_r(RSeedArgs a) {
    __shared__ float sc_s[4][NT * 64];
    __shared__ uint16_t qh_s[4][32 * NC];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = lane >> 4, cj = lane & 15;
    const int64_t q = (int64_t)blockIdx.x * 4 + w;
    if (q >= a.nq) return;  // (no workgroup barrier below)
    const int centred = M == LIRA_METRIC_L2 ? 1 : 2;
    const bool samp = a.work && (q & 7) == 0;
    const int64_t pair0 = q * a.nprobe;
    const int p0raw = a.probe[pair0];
    const int p0 = p0raw >= 0 && p0raw < a.n_lists ? p0raw : -1;
    const int tile0 = p0 >= 0 ? a.tile_off[p0] : 0, ntl = p0 >= 0 ? a.tile_off[p0 + 1] - tile0 : 0;
    // the first seed tile's B fragments and every tile's xadj, requested first (their
    // latency overlaps the record below); tiles past the list's end repeat its first
    const int64_t tile_bytes = a.dpad * 64 * 4;
    const uint32_t lane_off = (uint32_t)((g >> 1) * 4096 + (g & 1) * 1024 + cj * 16);
    rbf16x8 Bc[NC][4], Bn[NC][4];
    rf4 xa[NT];
    auto load_tile = [&](int t, rbf16x8 (&Bt)[NC][4]) {
        const int tt = tile0 + (t < ntl ? t : 0);
        const char *base = a.Xb + (int64_t)tt * tile_bytes + lane_off;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i) Bt[c][i] = *(const rbf16x8 *)(base + c * 8192 + i * 256);
    };
    if (ntl > 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) xa[t] = *(const rf4 *)(a.xadj + (int64_t)(tile0 + (t < ntl ? t : 0)) * 64 + 4 * cj);
        load_tile(0, Bc);
    }
    // slot 0's record, all 64 lanes (pair_record's values: q' = fl(q - c) (L2) or q,
    // double sums; no filter -- the seed's own list), its hi parts kept in LDS for the A operand
    float qv = 0.0f, qnorm = 0.0f, qres = 0.0f;
    if (p0 >= 0) {
        const float *qr = a.Q + q * a.d, *pv = a.pivot + (int64_t)p0 * a.d;
        double s2 = 0.0, t2 = 0.0, e2 = 0.0;
#pragma unroll
        for (int r = 0; r < NC / 2 + 1; ++r) {
            const int64_t j = lane + 64 * r;
            if (j < 32 * NC) {
                float x = 0.0f, cv = 0.0f;
                if (j < a.d) {
                    x = qr[j];
                    cv = pv[j];
                }
                const float sv = M == LIRA_METRIC_L2 ? x - cv : x;
                const uint32_t h = bf16_rne_sat(sv);
                qh_s[w][j] = (uint16_t)h;
                a.QH[pair0 * a.dpad + j] = (uint16_t)h;
                if (j < a.d) {
                    s2 = __builtin_fma((double)sv, (double)sv, s2);
                    const double rr = (double)(sv - __uint_as_float(h << 16));
                    e2 = __builtin_fma(rr, rr, e2);
                    if (M == LIRA_METRIC_L2) {
                        const double df = (double)x - (double)cv;
                        t2 = __builtin_fma(df, df, t2);
                    } else {
                        t2 = __builtin_fma((double)x, (double)cv, t2);
                    }
                }
            }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            s2 += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, s2), m));
            t2 += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, t2), m));
            e2 += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, e2), m));
        }
        const float qnu = __double2float_ru(__builtin_sqrt(s2) * (1.0 + 0x1p-40));
        const float dq = M == LIRA_METRIC_L2 ? (float)__builtin_sqrt(t2) : (float)t2;
        qv = M == LIRA_METRIC_L2 ? (float)s2 : dq;
        qnorm = qnu;
        qres = __double2float_ru(__builtin_sqrt(e2) * (1.0 + 0x1p-40));
        if (lane == 0) {
            a.QN[pair0] = make_float4(qv, qnu, __int_as_float((int)pair0), dq);
            a.QE[pair0] = qres;
            if (a.pqn) a.pqn[pair0] = qnu;
        }
    }
    if (lane == 0) a.probe_live[pair0] = p0raw;
    int est = 0;
    if (samp && lane < 16 && p0 >= 0) est = (a.list_size[p0] + 255) / 256;  // (slot 0: its whole list, lane 0 counts)
    if (lane != 0) est = 0;
    float T = __builtin_inff();
    if (ntl > 0) {  // (an empty list: no bound)
        // the screened tiles' largest radius and hi residual (errE_r is monotone in both)
        float rb = 0.0f, hr = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (t < ntl) {
                rb = fmaxf(rb, a.tstat[tile0 + t].y);
                hr = fmaxf(hr, a.tres ? a.tres[tile0 + t] : 0.0f);
            }
        }
        const float Rb = fminf(a.rmax[p0], rup(rb));
        const float Rx = M == LIRA_METRIC_IP ? a.rmaxx[p0] : 0.0f;
        const float E = errE_r<M>(qnorm, Rb, a.tres ? hr : -1.0f, qres, (float)a.dpad, qv, Rx, (float)a.d);
        // A: row 0 = hi(q'), dims 32 c + 8 g .. + 7 in lane (g, 0), the other rows zero
        __builtin_amdgcn_wave_barrier();
        rbf16x8 A[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (cj == 0) v = *(const uint4 *)&qh_s[w][32 * c + 8 * g];
            A[c] = __builtin_bit_cast(rbf16x8, v);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (t + 1 < NT) load_tile(t + 1, Bn);  // (the next tile's loads under this one's MFMAs)
            rf4 acc[4];
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[c], Bc[c][i], c == 0 ? (rf4)(-xa[t][i]) : acc[i],
                                                                     0, 0, 0);
            if (t + 1 < NT) {
#pragma unroll
                for (int c = 0; c < NC; ++c)
#pragma unroll
                    for (int i = 0; i < 4; ++i) Bc[c][i] = Bn[c][i];
            }
            // row 0 (lanes 0..15, register 0): candidate 4 cj + i of the tile
            if (g == 0)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float wv = acc[i][0];
                    const float sc = M == LIRA_METRIC_L2 ? qv - 2.0f * wv : -(wv + qv);
                    sc_s[w][t * 64 + 4 * cj + i] = t < ntl && sc == sc ? sc : __builtin_inff();
                }
        }
        __builtin_amdgcn_wave_barrier();
        u64 key[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) key[t] = ((u64)f2ord(sc_s[w][t * 64 + lane]) << 32) | (uint32_t)(t * 64 + lane);
        wave_sort<NT>(key);
        const u64 kk = wave_list_at<NT>(key, a.k - 1);
        const float sk = key_score(kk);
        if (sk < 3e38f)
            T = M == LIRA_METRIC_L2 ? __double2float_ru(bound_P<LIRA_METRIC_L2>((double)sk, (double)E, (double)a.d))
                                    : __double2float_ru(bound_P<LIRA_METRIC_IP>((double)sk, (double)E, (double)a.d));
    }
    const uint32_t qb = T < 3e38f ? f2ord(T) : ~0u;
    if (lane == 0) a.qbound[q] = qb;
    // slots 1.. under the bound (the partition filter)
    for (int s0 = 1; a.records && s0 < a.nprobe; s0 += 4) {
        const int slot = s0 + (lane >> 4);
        const bool valid = slot < a.nprobe;
        const int64_t pair = pair0 + (valid ? slot : 0);
        const int praw = valid ? a.probe[pair] : -1;
        est += pair_record(a.Q, a.d, pair, valid, praw, a.nprobe, a.n_lists, a.pivot, centred, a.lstat, qb,
                           a.probe_live, a.QN, a.QE, a.pqn, a.QH, a.dpad, samp ? a.list_size : nullptr, a.lsamp,
                           a.rmaxx);
    }
    if (samp) {  // lanes 0, 16, 32, 48 hold their pair groups' sums
        const int tot = __builtin_amdgcn_readlane(est, 0) + __builtin_amdgcn_readlane(est, 16) +
                        __builtin_amdgcn_readlane(est, 32) + __builtin_amdgcn_readlane(est, 48);
        if (lane == 0 && tot) atomicAdd(a.work + ((q >> 3) & 63), (unsigned)tot);
    }
}

template <int NC, int M>
static hipError_t launch_seed_rn(const RSeedArgs &a, int nt, hipStream_t st) {
    const dim3 g((unsigned)((a.nq + 3) / 4)), b(256);
    if (nt == 1) hipLaunchKernelGGL((k_seed_r<NC, M, 1>), g, b, 0, st, a);
    else if (nt == 2) hipLaunchKernelGGL((k_seed_r<NC, M, 2>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_seed_r<NC, M, 4>), g, b, 0, st, a);
    return hipGetLastError();
}
template <int M>
static hipError_t launch_seed_rm(const RSeedArgs &a, int nt, hipStream_t st) {
    switch (a.dpad / 32) {
        case 1: return launch_seed_rn<1, M>(a, nt, st);
        case 2: return launch_seed_rn<2, M>(a, nt, st);
        case 3: return launch_seed_rn<3, M>(a, nt, st);
        case 4: return launch_seed_rn<4, M>(a, nt, st);
        default: return hipErrorInvalidValue;
    }
}
hipError_t launch_seed_r(const RSeedArgs &a, int nt, hipStream_t st) {
    if (a.nq <= 0) return hipSuccess;
    if (nt != 1 && nt != 2 && nt != 4) return hipErrorInvalidValue;
    return a.metric == LIRA_METRIC_L2 ? launch_seed_rm<LIRA_METRIC_L2>(a, nt, st)
                                      : launch_seed_rm<LIRA_METRIC_IP>(a, nt, st);
}

bool rscreen_shape_ok(int64_t dpad, int64_t k) {
    return k >= 1 && k <= 120 && dpad >= 32 && dpad % 32 == 0 && (dpad <= 128 || (dpad % 64 == 0 && dpad <= 4096));
}
int rscreen_smem(int rl, int waves) {
    return rl == 1 ? RSmem<1, 4>::total : rl == 2 ? RSmem<2, 4>::total : waves == 8 ? RSmem<4, 8>::total : RSmem<4, 4>::total;
}
int rscreen_qr(int rl, int waves) {
    return rl == 1 ? RSmem<1, 4>::QR : rl == 2 ? RSmem<2, 4>::QR : waves == 8 ? RSmem<4, 8>::QR : RSmem<4, 4>::QR;
}

template <int NC, int M, int RL, int W>
static hipError_t launch_r(const RArgs &a, int grid, hipStream_t st) {
    static std::atomic<uint64_t> attr{0};
    hipError_t e = set_smem_attr_once(attr, (const void *)k_screen_r<NC, M, RL, W>, RSmem<RL, W>::total);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_screen_r<NC, M, RL, W>), dim3(grid), dim3(64 * W), (RSmem<RL, W>::total), st, a);
    return hipGetLastError();
}

template <int M, int RL, int W>
static hipError_t launch_rm(const RArgs &a, int grid, hipStream_t st) {
    switch (a.dpad / 32) {
        case 1: return launch_r<1, M, RL, W>(a, grid, st);
        case 2: return launch_r<2, M, RL, W>(a, grid, st);
        case 3: return launch_r<3, M, RL, W>(a, grid, st);
        case 4: return launch_r<4, M, RL, W>(a, grid, st);
        default:
            if (a.dpad % 64 == 0 && a.dpad <= 4096) return launch_r<0, M, RL, W>(a, grid, st);  // (streamed A)
            return hipErrorInvalidValue;
    }
}

template <int M>
static hipError_t launch_rmm(const RArgs &a, int rl, int waves, int grid, hipStream_t st) {
    if (rl == 1) return launch_rm<M, 1, 4>(a, grid, st);
    if (rl == 2) return launch_rm<M, 2, 4>(a, grid, st);
    if (rl == 4) return waves == 8 ? launch_rm<M, 4, 8>(a, grid, st) : launch_rm<M, 4, 4>(a, grid, st);
    return hipErrorInvalidValue;
}

hipError_t launch_rscreen(const RArgs &a, int rl, int waves, int grid, hipStream_t st) {
    return a.metric == LIRA_METRIC_L2 ? launch_rmm<LIRA_METRIC_L2>(a, rl, waves, grid, st)
                                      : launch_rmm<LIRA_METRIC_IP>(a, rl, waves, grid, st);
}

}  // namespace lira
