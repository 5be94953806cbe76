// lira_wscreen.hip -- the wide screen (gfx950): 256 query rows per work item,
// one 512-thread workgroup per CU, v_mfma_f32_32x32x16_bf16 on the hi parts
// of the pivot-centred vectors, rigorous bound + exact re-check in k_smerge.
// Replaces search.cpp:468-493 (the per-query candidate loop over the probed
// buckets) for L2, k <= 24, dpad <= 256; results identical to the all-exact
// scan (lira_scan.hip k_scan).  The error model is k_screen_m<..., 3>'s
// (lira_bounds.hpp err_E, split = 3): only the staging and the MFMA shape
// differ.
//
// Why a second screen.  k_screen_m (64 rows per item, 2 workgroups per CU)
// stages every candidate chunk through LDS for 64 query rows: 4 KiB of L2 ->
// LDS traffic per 64 x 32-dim MFMA tile set, so on latent data (nothing
// pruned) it ran at ~6 TB/s of staging and 0.17 of HBM peak, waiting.  Here
// a staged chunk feeds 256 rows (8 waves x 32), the queries' hi parts sit in
// registers for the whole item (no query staging at all), and the per-pair
// constants come from k_pairs (no k_qstage).
//
// Work item: (virtual partition, block of <= 256 pairs, chunk of the bucket),
// k_plan's XCD-ordered table.  A block is 128 candidates (2 tiles); the ring
// holds NS slots of 4 k-steps (64 dims) x 2 tiles of Xb hi parts (16 KiB).
//
// Schedule.  Wave 0 is also the scheduler: one step ahead of the DMA issue it
// writes the next slot's entry (item, block, slot in block, block radius
// range) into an LDS ring, skipping blocks whose radius range lies outside
// every row's triangle-inequality interval (stale intervals are wider: safe).
// Every slot: each wave waits for its own LDS-DMA pieces of that slot
// (counted vmcnt), one workgroup barrier, each wave issues its pieces of the
// slot NS-1 ahead, then computes.  Item transitions happen at the same slot
// in every wave, so the barriers stay aligned.
//
// MFMA layout (v_mfma_f32_32x32x16_bf16, cdna_hip_programming.md section 3):
// A = 32 query rows x 16 dims (lane l: row l & 31, dims 8 (l >> 5) ..), from
// registers; B = 16 dims x 32 candidates (lane l: candidate column l & 31),
// one ds_read_b128 from Xb's hi pieces ([h 2][p 64][8 bf16] per tile and
// 16-dim chunk, candidate row 4 (p & 15) + (p >> 4)); D: lane l holds
// candidate column l & 31 for rows (reg & 3) + 8 (reg >> 2) + 4 (l >> 5).
// Per block and wave: 4 column groups (2 tiles x 2 halves) = 4 accumulators.
#include <algorithm>
#include <atomic>
#include <string>

#include "lira_bounds.hpp"
#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
typedef float wf32x16 __attribute__((ext_vector_type(16)));

static constexpr int kWQR = 256;    // query rows per item
static constexpr int kWNW = 8;      // waves (32 rows each)
static constexpr int kWK2 = 32;     // row list keys (k <= 24)
static constexpr int kWBH = 8;      // survivor buffer keys per (row, half-wave): 16 per row
static constexpr int kWNS = 3;      // ring slots
static constexpr int kWSlot = 16384;  // 4 k-steps x 2 tiles x 2 KiB
static constexpr int kWMaxBlk = 128;  // blocks (of 128 candidates) per item

struct WSmem {
    static constexpr int ring = 0;
    static constexpr int xad = ring + kWNS * kWSlot;        // [NS][128] f32: a block's xadj in B-fragment order
    static constexpr int lists = xad + 4 * 512;             // [256][K2] u64
    static constexpr int bufs = lists + kWQR * kWK2 * 8;    // [256][2][BH] u64: survivor half-buffers
    static constexpr int irec = bufs + kWQR * 2 * kWBH * 8;  // [4][8] int: item records (k_wrec)
    static constexpr int total = irec + 4 * 32;
};
static_assert(WSmem::total <= 160 * 1024, "k_screen_w LDS");

struct WArgs {
    const uint16_t *Xb;
    const float *xadj;   // centred (xadjc)
    const float *rmax;   // centred (rmaxc)
    const int32_t *tile_off, *cnt, *qoff, *qlist;
    const int4 *itab, *wrec;  // (wrec: k_wrec's per-item records, 2 int4 each)
    int32_t *head;
    const float *Q, *pivot;
    const float4 *QN;    // per pair: qn, qnorm (up), -, ||q - c|| (k_pairs)
    const float *QE;     // per pair: ||q' - hi(q')|| (up)
    const float2 *tstat;
    const float *tres;
    u64 *partial;
    float *pE;
    uint32_t *qbound;
    int64_t d, dpad;
    int n_lists, n_virt, nprobe, k, bpc, bpc_near, nch_max, share, tri;
    unsigned long long *stats;
};

// ---- per-pair records + the partition filter (lira_bounds.hpp pair_record) ----
// One pair per 16 lanes, the filter bound from qbound (k_seed_t's seed); the
// default L2 screen runs the same records inside k_seed_t<..., PAIRS> instead.
__global__ __launch_bounds__(256) void k_pairs(const float *Q, int64_t d, const int32_t *probe, int64_t npairs,
                                               int nprobe, int n_lists, const float *pivot, int centred,
                                               const float2 *lstat, const uint32_t *qbound, int32_t *probe_live,
                                               float4 *QN, float *QE, float *pqn, uint16_t *QH, int64_t dpad) {
    const int64_t pair = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const bool valid = pair < npairs;
    const int praw = valid ? probe[pair] : -1;
    const uint32_t qb = valid && lstat && qbound ? qbound[pair / nprobe] : ~0u;
    pair_record(Q, d, pair, valid, praw, nprobe, n_lists, pivot, centred, lstat && qbound ? lstat : nullptr, qb,
                probe_live, QN, QE, pqn, QH, dpad);
}

// ---- the wide screen ----------------------------------------------------------
__device__ __forceinline__ void wdma16(const void *gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_addr)
        : "memory");
}
__device__ __forceinline__ void wdma4(const void *gsrc, uint32_t lds_addr) {  // 4 B per lane
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_addr)
        : "memory");
}
__device__ __forceinline__ void wait_vm(int n) {  // s_waitcnt vmcnt(n), n <= 7 (uniform)
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    }
}
// fp32 bounds with explicit margins (the refresh runs once per block and row; the
// double-precision forms of lira_bounds.hpp cost ~2k cycles per block there).
// up(x) / dn(x): applied to the round-to-nearest result x of one fp32 operation,
// a value >= / <= its exact result (x +- |x| 2^-22 covers the 2^-24 rounding of
// the operation and of this fma itself, either sign).
__device__ __forceinline__ float wup(float x) { return __builtin_fmaf(__builtin_fabsf(x), 0x1p-22f, x); }
__device__ __forceinline__ float wdn(float x) { return __builtin_fmaf(-__builtin_fabsf(x), 0x1p-22f, x); }
// err_E<L2>(qnorm, Rb, d, split = 3, dpad, centred = 1, hres, qres) as an fp32 upper
// bound: every term is non-negative, so ~16 round-to-nearest operations stay within
// 16 2^-24 relative and the final (1 + 2^-17) covers them; the constants are rounded
// up (1.0002 for 1.0001, 1.03 for 1.02, 10.5 for 8.4 + 2.01, 2^-126 for d 2^-140)
__device__ __forceinline__ float werr_E(float qnorm, float Rb, float dpf, float hres, float qres) {
    const float ex = hres >= 0.0f ? hres * 1.0002f : 0x1p-8f * 1.03f * Rb;
    const float re = Rb + ex;
    const float ed = ex * qnorm + qres * re * 1.0002f + 2.0f * dpf * 0x1p-22f * 1.03f * qnorm * re +
                     2.0f * dpf * 0x1p-96f * (qnorm + re + 1.0f);
    const float s = qnorm + Rb;
    return wup((2.0f * ed + 10.5f * 0x1p-24f * s * s + 0x1p-126f) * (1.0f + 0x1p-17f));
}

__device__ __forceinline__ int wxcd_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 7u);
}
// ---- per-item records of the wide screen (one thread per item of k_plan's table) ----
// 0 p, 1 chunk, 2 first pair index into qlist, 3 rows (pairs), 4 first tile (absolute),
// 5 tiles, 6 rmax bits, 7 blocks of 128 candidates
__global__ __launch_bounds__(256) void k_wrec(const int4 *itab, const int32_t *head, const int32_t *tile_off,
                                              const int32_t *qoff, const int32_t *cnt, const float *rmax,
                                              int n_lists, int n_virt, int bpc, int bpc_near, int4 *wrec) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= head[18]) return;
    const int4 e = itab[i];
    const int vp = e.x, qb = e.y, ch = e.z;
    const int p = vp >= n_lists ? vp - n_lists : vp;
    const int tile0 = tile_off[p], ntl = tile_off[p + 1] - tile0;
    const int b = vp < n_lists && n_virt > n_lists ? bpc_near : bpc;
    const int tbb = ch * b * 4, tbe = min(ntl, tbb + b * 4);
    wrec[2 * i] = make_int4(p, ch, qoff[vp] + qb * kWQR, min(kWQR, cnt[vp] - qb * kWQR));
    wrec[2 * i + 1] = make_int4(tile0 + tbb, tbe - tbb, __float_as_int(rmax[p]), (tbe - tbb + 1) / 2);
}

#ifdef LIRA_WCLOCKS
static constexpr bool kWClk = true;  // timing build (tools/wclocks.py): phase cycles into the stats words
#else
static constexpr bool kWClk = false;
#endif

// A slot cursor: every wave advances it identically (uniform values).
struct WCur {
    int seq, blk, j;           // item sequence number (-1: past the end), block, slot in block
    int tfirst, ntiles, nblk;  // the item's first tile, tiles, blocks
};

template <int NKS>
__global__ __launch_bounds__(512, 1) void k_screen_w(WArgs a) {
    constexpr int NSL = (NKS + 3) / 4;  // ring slots per block
    // (a block's xadj sits at its first slot's ring position until it is re-issued,
    // NS - 1 slots later: the selection at its last slot reads it in time for NSL <= 2)
    static_assert(NSL <= 2, "k_screen_w: dpad <= 128");
    constexpr int SW = kWNW - 1;        // the item-claiming wave (the last rows: often empty)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const float *xads = (const float *)(smem + WSmem::xad);
    u64 *lists = (u64 *)(smem + WSmem::lists);
    u64 *bufs = (u64 *)(smem + WSmem::bufs);
    int *irec = (int *)(smem + WSmem::irec);
    __shared__ int xq[9], cl[2];
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)smem;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rl = lane & 31, hf = lane >> 5;
    const int k = a.k;
    const double dd = (double)a.d;
    unsigned long long *const cnt = kWClk ? nullptr : a.stats;
    long long ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t0 = 0, t1 = 0;  // (kWClk) phase cycles
    auto tick = [&](int slot) {
        if (kWClk) {
            const long long t = clock64();
            ck[slot] += t - t1;
            t1 = t;
        }
    };

    // ---------------- items: wave SW claims them and writes their records ----------------
    // irec[s & 3] = record of item sequence number s (8 ints; p = -1: no more items).
    // Record s + 1 is written when the issue cursor enters item s, so it is in LDS
    // one barrier before any cursor needs it; a record is overwritten four items
    // later, when both cursors have left it (the consume cursor trails by NS - 1 slots).
    auto claim = [&]() -> int {  // lane 0: the next item of this XCD's queue, stealing when empty
        int x = cl[0], tries = cl[1], it = -1;
        while (tries < 8) {
            const int i = xq[x] + atomicAdd(&a.head[2 + x], 1);
            if (i < xq[x + 1]) {
                it = i;
                break;
            }
            x = (x + 1) & 7;
            ++tries;
        }
        cl[0] = x;
        cl[1] = tries;
        return it;
    };
    auto write_rec = [&](int s) {  // wave SW
        if (lane == 0) {
            const int it = claim();
            int4 r0 = make_int4(-1, 0, 0, 0), r1 = make_int4(0, 0, 0, 0);
            if (it >= 0) {
                r0 = a.wrec[2 * it];
                r1 = a.wrec[2 * it + 1];
            }
            int4 *dst = (int4 *)(irec + (s & 3) * 8);
            dst[0] = r0;
            dst[1] = r1;
        }
        __builtin_amdgcn_wave_barrier();
    };
    auto load_item = [&](WCur &c, int s) {  // the cursor enters item s (its record is in irec)
        const int *R = irec + (s & 3) * 8;
        c.seq = __builtin_amdgcn_readfirstlane(R[0]) < 0 ? -1 : s;
        c.blk = 0;
        c.j = 0;
        c.tfirst = __builtin_amdgcn_readfirstlane(R[4]);
        c.ntiles = __builtin_amdgcn_readfirstlane(R[5]);
        c.nblk = __builtin_amdgcn_readfirstlane(R[7]);
    };
    auto advance = [&](WCur &c) -> bool {  // true when it entered a new item
        if (c.seq < 0) return false;
        if (++c.j < NSL) return false;
        c.j = 0;
        if (++c.blk < c.nblk) return false;
        load_item(c, c.seq + 1);
        return c.seq >= 0;
    };

    // ---------------- DMA issue of the slot at cursor c into ring position pos ----------------
    // wave w moves pieces 2w, 2w + 1 (k-step s = pc >> 2, tile pc >> 1 & 1, half pc & 1);
    // at a block's first slot wave 0 also moves the block's xadj in B-fragment
    // order p (one dword per lane: candidate 4 (p & 15) + (p >> 4) of the tile)
    // into xadj buffer pos.  Returns the DMA instructions issued.
    const int nkc = (int)(a.dpad / 16);  // 16-dim chunks of a tile in Xb
    auto issue = [&](const WCur &c, int pos) -> int {
        if (c.seq < 0) return 0;
        const int tba = c.tfirst + 2 * c.blk, ntv = min(2, c.ntiles - 2 * c.blk);
        const uint32_t slot = lds0 + WSmem::ring + (uint32_t)(pos * kWSlot);
        int n = 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int pc = 2 * wave + u, s = pc >> 2, T = (pc >> 1) & 1, h = pc & 1;
            const int ks = 4 * c.j + s;
            if (ks < NKS) {
                const uint16_t *src = a.Xb + ((int64_t)(tba + min(T, ntv - 1)) * nkc + ks) * 2048 + h * 512 + lane * 8;
                wdma16(src, slot + (uint32_t)((s * 2 + T) * 2048 + h * 1024));
                ++n;
            }
        }
        if (c.j == 0 && wave == 0) {
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                const float *src = a.xadj + (int64_t)(tba + min(T, ntv - 1)) * kTile + 4 * (lane & 15) + (lane >> 4);
                wdma4(src, lds0 + WSmem::xad + (uint32_t)(pos * 512 + T * 256));
                ++n;
            }
        }
        return n;
    };

    // ---------------- consumer state (wave w: rows 32 w + (lane & 31)) ----------------
    // D layout (A = candidates, B = queries): lane l holds the row 32 w + (l & 31)
    // and, per column group cg (tile cg >> 1, half cg & 1), the 16 candidates
    // p = 32 (cg & 1) + (reg & 3) + 8 (reg >> 2) + 4 (l >> 5) of the tile.
    int c_ch = 0;
    float c_R = 0.0f;
    int my_pair = -1, my_q = -1;
    float my_qn = 0.0f, my_qnorm = 0.0f, my_qres = 0.0f, my_dq = 0.0f, E_run = 0.0f, h_l = 0.0f;
    uint32_t pub = ~0u, own_pub = ~0u;
    float T_c = -1.0f, A_c = 0.0f;  // the row's bound T and its s_lim term A = (T + dl) / F (up)
    float2 ab_c = make_float2(-__builtin_inff(), __builtin_inff());
    wbf16x8 Aq[NKS];
    int b_tba = 0, b_ntv = 0, b_xb = 0, bcl = 0;  // bcl: keys in this lane's half-buffer of its row
    // kernel constants (double -> fp32, rounded up): bound_P's factor (1 + (d+4) u)(1 + 2^-50)
    // with slack, and 1 / F, F = 1 - (d+4) u (s_lim, the skip radius)
    const float Gp = __double2float_ru((1.0 + (dd + 4.0) * kU) * (1.0 + 0x1p-40));
    const float iF = __double2float_ru((1.0 / (1.0 - (dd + 4.0) * kU)) * (1.0 + 0x1p-40));
    const float dpf = (float)a.dpad;
    // bound_P<L2>(sk, E) as an fp32 upper bound
    auto bndP = [&](float sk, float E) { return wup(wup(wup(sk + E) * Gp) + 0x1p-126f); };
    bool wdead = true;
    wf32x16 acc[4];
    float bl_lo[2], bl_hi[2], bl_re[2];  // the item's blocks b = lane, lane + 64: radius range, hi residual
    const int my_row = wave * 32 + rl;

    // the row's skip interval [A, B] for ||x - c|| from bound T (k_screen_m's refresh:
    // rad = sqrt((T + dl) / F) (1 + 2^-40), A = ||q - c|| (1 - 2^-22) - rad, B = .. + rad),
    // in fp32 rounded outward; A_c (s_lim's T term) alongside
    auto interval = [&](float T) {
        float2 ab = make_float2(-__builtin_inff(), __builtin_inff());
        A_c = wup(wup(fmaxf(T, 0.0f) + 0x1p-126f) * iF);
        if (my_pair < 0) {
            ab = make_float2(__builtin_inff(), -__builtin_inff());
        } else if (T < 3e38f && iF < 2.0f) {
            const float rad = wup(wup(sqrtf(A_c)) * (1.0f + 0x1p-20f));
            ab = make_float2(wdn(wdn(my_dq * (1.0f - 0x1p-21f)) - rad), wup(wup(my_dq * (1.0f + 0x1p-21f)) + rad));
        }
        return ab;
    };

    // merge the half-buffers of the rows in `rows` (bit r: row 32 w + r) into
    // their lists, two rows per half-wave network pass; their counts restart
    auto flush_rows = [&](uint32_t rows) {
        const uint32_t all = rows;
        while (rows) {
            const int ra = __builtin_ctz(rows);
            rows &= rows - 1;
            int rb = ra;
            if (rows) {
                rb = __builtin_ctz(rows);
                rows &= rows - 1;
            }
            const int r = hf ? rb : ra;  // this half's row
            const int RR = wave * 32 + r;
            const int n0 = __builtin_amdgcn_readlane(bcl, ra), n1 = __builtin_amdgcn_readlane(bcl, ra + 32);
            const int m0 = __builtin_amdgcn_readlane(bcl, rb), m1 = __builtin_amdgcn_readlane(bcl, rb + 32);
            const int c0 = hf ? m0 : n0, c1 = hf ? m1 : n1;
            u64 lst[1] = {lists[RR * kWK2 + rl]};
            const int hb = rl >> 3, e = rl & 7;
            const u64 b = rl < 16 && e < (hb ? c1 : c0) ? bufs[(RR * 2 + hb) * kWBH + e] : kEmptyKey;
            half_merge_batch1<1>(lst, b);
            lists[RR * kWK2 + rl] = lst[0];  // (one row: both halves write the same keys)
            __builtin_amdgcn_wave_barrier();
        }
        if ((all >> rl) & 1u) bcl = 0;
    };

    auto prologue = [&](int s) {
        const int *R = irec + (s & 3) * 8;
        const int p = __builtin_amdgcn_readfirstlane(R[0]), pbase = __builtin_amdgcn_readfirstlane(R[2]);
        const int nval = __builtin_amdgcn_readfirstlane(R[3]);
        c_ch = __builtin_amdgcn_readfirstlane(R[1]);
        c_R = __int_as_float(__builtin_amdgcn_readfirstlane(R[6]));
        my_pair = my_row < nval ? a.qlist[pbase + my_row] : -1;
        my_q = my_pair >= 0 ? my_pair / a.nprobe : -1;
        float4 qr = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float qe = 0.0f;
        pub = ~0u;
        if (my_pair >= 0) {
            qr = a.QN[my_pair];
            qe = a.QE[my_pair];
            if (a.qbound) pub = __hip_atomic_load(a.qbound + my_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        my_qn = qr.x;
        my_qnorm = qr.y;
        my_dq = qr.w;
        my_qres = qe;
        own_pub = ~0u;
        E_run = 0.0f;
        T_c = -1.0f;  // (no bound cached yet)
        bcl = 0;
        // the row's hi parts of fl(q - c), 8 dims per lane per 16-dim k-step
        const float *qrow = my_pair >= 0 ? a.Q + (int64_t)my_q * a.d : nullptr;
        const float *pv = a.pivot + (int64_t)p * a.d;
#pragma unroll
        for (int s2 = 0; s2 < NKS; ++s2) {
            const int64_t j0 = 16 * s2 + 8 * hf;
            uint32_t w4[4];
            if (qrow && j0 + 8 <= a.d && (a.d & 3) == 0) {
                const float4 x0 = *(const float4 *)(qrow + j0), x1 = *(const float4 *)(qrow + j0 + 4);
                const float4 c0 = *(const float4 *)(pv + j0), c1 = *(const float4 *)(pv + j0 + 4);
                w4[0] = bf16_rne_sat(x0.x - c0.x) | (bf16_rne_sat(x0.y - c0.y) << 16);
                w4[1] = bf16_rne_sat(x0.z - c0.z) | (bf16_rne_sat(x0.w - c0.w) << 16);
                w4[2] = bf16_rne_sat(x1.x - c1.x) | (bf16_rne_sat(x1.y - c1.y) << 16);
                w4[3] = bf16_rne_sat(x1.z - c1.z) | (bf16_rne_sat(x1.w - c1.w) << 16);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    uint32_t pr[2];
#pragma unroll
                    for (int f = 0; f < 2; ++f) {
                        const int64_t jj = j0 + 2 * e + f;
                        pr[f] = qrow && jj < a.d ? bf16_rne_sat(qrow[jj] - pv[jj]) : 0u;
                    }
                    w4[e] = pr[0] | (pr[1] << 16);
                }
            }
            Aq[s2] = __builtin_bit_cast(wbf16x8, make_uint4(w4[0], w4[1], w4[2], w4[3]));
        }
        // the item's block radius ranges / hi residuals into registers (no global
        // load inside the block loop: its wait would drain the DMA ring)
        const int tfirst = __builtin_amdgcn_readfirstlane(R[4]), ntiles = __builtin_amdgcn_readfirstlane(R[5]);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int b = lane + 64 * u;
            float lo = -__builtin_inff(), hi = __builtin_inff(), re = -1.0f;
            if (2 * b < ntiles) {
                const int t = tfirst + 2 * b;
                const bool two = 2 * b + 1 < ntiles;
                if (a.tstat) {
                    const float2 s0 = a.tstat[t], s1 = two ? a.tstat[t + 1] : s0;
                    lo = fminf(s0.x, s1.x);
                    hi = fmaxf(s0.y, s1.y);
                }
                if (a.tres) re = two ? fmaxf(a.tres[t], a.tres[t + 1]) : a.tres[t];
            }
            bl_lo[u] = lo;
            bl_hi[u] = hi;
            bl_re[u] = re;
        }
        u64 *L = lists + (wave * 32) * kWK2;
        for (int i = lane; i < 32 * kWK2; i += 64) L[i] = kEmptyKey;
        ab_c = interval(pub != ~0u ? ord2f(pub) : __builtin_inff());
        __builtin_amdgcn_wave_barrier();
    };

    auto epilogue = [&]() {
        const u64 pend = __ballot(bcl > 0);
        flush_rows((uint32_t)pend | (uint32_t)(pend >> 32));
        for (int r = 0; r < 32; r += 2) {  // lists out, two rows per store round
            const int rr = r + hf, pr = __shfl(my_pair, rr, 64);
            if (pr >= 0)
                a.partial[((int64_t)pr * a.nch_max + c_ch) * kWK2 + rl] = lists[(wave * 32 + rr) * kWK2 + rl];
        }
        if (lane < 32 && my_pair >= 0) {
            if (a.pE) a.pE[(int64_t)my_pair * a.nch_max + c_ch] = fmaxf(E_run, 0x1p-126f);
            if (a.qbound) {
                const u64 kk = lists[my_row * kWK2 + k - 1];
                if (kk != kEmptyKey) atomicMin(a.qbound + my_q, f2ord(bndP(key_score(kk), E_run)));
            }
        }
    };

    // block start: the row's dot threshold h_l for this block; wdead when no
    // row of the wave can use the block (triangle inequality, or no pairs)
    auto refresh = [&](float b_lo, float b_hi, float b_re) {
        const u64 kk = lists[my_row * kWK2 + k - 1];
        float T = kk == kEmptyKey ? __builtin_inff() : bndP(key_score(kk), E_run);
        if (a.share && a.qbound && my_pair >= 0 && kk != kEmptyKey && lane < 32) {
            const uint32_t b = f2ord(T);
            if (b < own_pub) {
                atomicMin(a.qbound + my_q, b);
                own_pub = b;
            }
        }
        if (pub != ~0u) T = fminf(T, ord2f(pub));
        if (T != T_c) {  // (the row's bound moved)
            T_c = T;
            ab_c = interval(T);
        }
        const float Rb = a.tri ? fminf(c_R, wup(b_hi * (1.0f + 0x1p-19f))) : c_R;
        const float Eb = werr_E(my_qnorm, Rb, dpf, b_re, my_qres);
        // row_h<L2>(lim = s_lim(T, Eb)): pass iff fl(dot - xadj) >= (qn - lim) / 2 - 1.05 u (|q| + Rb)^2,
        // rounded down with a margin for this fp32 evaluation
        const float lim = wup(A_c + Eb);
        const float sq = wup((my_qnorm + Rb) * (my_qnorm + Rb));
        const float c = wup(1.06f * 0x1p-24f * sq);
        const float h0 = (my_qn - lim) * 0.5f - c;
        h_l = my_pair < 0 ? __builtin_inff() : h0 - (__builtin_fabsf(my_qn) + lim + c) * 0x1p-21f;
        E_run = fmaxf(E_run, Eb);
        wdead = !__any(my_pair >= 0) || (a.tri && __all(b_hi < ab_c.x || b_lo > ab_c.y));
    };

    // ---------------- selection of one block: lane = row, 64 candidates per lane ----------------
    auto select_cg = [&](auto cgc) {
        constexpr int cg = decltype(cgc)::value, T = cg >> 1, tp = cg & 1;
        if (T >= b_ntv) return;  // (uniform: past the list's end)
        const float hp = fmaxf(h_l, -3.40282347e38f);  // (padding: xadj = +inf never passes)
        const float *xb = xads + b_xb * 128 + 4 * hf + T * 64 + 32 * tp;
        wf32x16 w;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 x4 = *(const float4 *)(xb + 8 * g);
            w[4 * g + 0] = acc[cg][4 * g + 0] - x4.x;
            w[4 * g + 1] = acc[cg][4 * g + 1] - x4.y;
            w[4 * g + 2] = acc[cg][4 * g + 2] - x4.z;
            w[4 * g + 3] = acc[cg][4 * g + 3] - x4.w;
        }
        float m = fmaxf(fmaxf(w[0], w[1]), w[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) m = fmaxf(fmaxf(m, w[r]), w[r + 1]);
        m = fmaxf(m, w[15]);
        if (!__any(m >= hp)) return;
        // the registers (candidates) some lane passes, then one uniform pass per such
        // register: a lane appends at most one key per pass, so a full half-buffer
        // is merged right before the append that would overflow it
        uint32_t rmask = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) rmask |= __any(w[r] >= hp) ? 1u << r : 0u;
        const uint32_t rbase = (uint32_t)(b_tba + T) * kTile + (uint32_t)(16 * hf + 2 * tp);
        u64 *mybuf = bufs + (size_t)(my_row * 2 + hf) * kWBH;
        while (rmask) {
            const int r = __builtin_ctz(rmask);
            rmask &= rmask - 1;
            const float wr = w[r], dv = acc[cg][r];
            const bool pass = wr >= hp;
            const u64 full = __ballot(pass && bcl == kWBH);
            if (full) flush_rows((uint32_t)full | (uint32_t)(full >> 32));
            if (pass) {
                // screened score fl(qn + 2 xadj) - 2 dot; storage row 4 (p & 15) + (p >> 4),
                // p = 32 tp + (r & 3) + 8 (r >> 2) + 4 hf
                const float sc = __builtin_fmaf(-2.0f, dv, my_qn + 2.0f * (dv - wr));
                mybuf[bcl] = ((u64)f2ord(sc) << 32) | (rbase + (uint32_t)(4 * ((r & 3) + 8 * ((r >> 2) & 1)) + (r >> 3)));
                ++bcl;
                if (cnt) atomicAdd(cnt + 7, 1ull);
            }
        }
    };
    auto select = [&]() {
        select_cg(std::integral_constant<int, 0>{});
        select_cg(std::integral_constant<int, 1>{});
        select_cg(std::integral_constant<int, 2>{});
        select_cg(std::integral_constant<int, 3>{});
        // rows whose half-buffer is full merge now (the next block may append)
        const u64 full = __ballot(bcl == kWBH);
        if (full) flush_rows((uint32_t)full | (uint32_t)(full >> 32));
    };

    // the MFMAs of slot J of the current block (ring position pos): A = the
    // candidates' fragments from LDS, B = the rows' registers
    const uint32_t loff = (uint32_t)(hf * 1024 + rl * 16);
    auto mfma_slot = [&](auto jc, int pos) {
        constexpr int J = decltype(jc)::value;
        constexpr int NS4 = NKS - 4 * J < 4 ? NKS - 4 * J : 4;
        const char *sb = smem + WSmem::ring + pos * kWSlot + loff;
        wbf16x8 bv[NS4][4];
#pragma unroll
        for (int s = 0; s < NS4; ++s)
#pragma unroll
            for (int cg = 0; cg < 4; ++cg)
                bv[s][cg] = *(const wbf16x8 *)(sb + (s * 2 + (cg >> 1)) * 2048 + (cg & 1) * 512);
#pragma unroll
        for (int s = 0; s < NS4; ++s)
#pragma unroll
            for (int cg = 0; cg < 4; ++cg)
                acc[cg] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bv[s][cg], Aq[4 * J + s], acc[cg], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // DS reads: k-steps 0, 1
#pragma unroll
        for (int s = 0; s < NS4; ++s) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMAs of k-step s
            if (s + 2 < NS4) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // reads of k-step s + 2
        }
    };

    // ---------------- the ring: issue cursor NS - 1 slots ahead of the consume cursor ----------------
    if (wave == SW && lane == 0) {
        for (int r = 0; r < 9; ++r) xq[r] = a.head[10 + r];
        cl[0] = wxcd_id();
        cl[1] = 0;
    }
    if (wave == SW) {
        __builtin_amdgcn_wave_barrier();
        write_rec(0);
        write_rec(1);
    }
    __syncthreads();
    WCur ic, cc;  // issue / consume cursors
    load_item(ic, 0);
    load_item(cc, 0);
    int np0 = issue(ic, 0), np1 = 0, np2 = 0;  // this wave's DMAs of positions 0, 1, 2
    if (advance(ic) && wave == SW) write_rec(ic.seq + 1);
    np1 = issue(ic, 1);
    int cur = -1;  // the item the rows hold
    if (kWClk) t0 = t1 = clock64();

#pragma unroll 1
    for (int n = 0;; ++n) {
        const int r = n % kWNS;
        wait_vm(r == 0 ? np1 : r == 1 ? np2 : np0);  // this wave's DMAs of slot n have landed
        __syncthreads();  // ... everyone's; position (n - 1) % 3 is free; the next record written
        tick(1);
        {
            const bool entered = advance(ic);  // slot n + 2 -> position (n + 2) % 3
            const int c = issue(ic, (r + 2) % kWNS);
            if (r == 0) np2 = c;
            else if (r == 1) np0 = c;
            else np1 = c;
            tick(2);
            if (entered && wave == SW) write_rec(ic.seq + 1);
            tick(7);
        }
        if (cc.seq < 0) {  // end of the items (every wave at the same slot)
            if (cur >= 0) epilogue();
            break;
        }
        if (cc.seq != cur) {  // item transition
            if (cur >= 0) epilogue();
            prologue(cc.seq);
            cur = cc.seq;
        }
        tick(3);
        const int j = cc.j;
        if (j == 0) {  // block start
            b_tba = cc.tfirst + 2 * cc.blk;
            b_ntv = min(2, cc.ntiles - 2 * cc.blk);
            b_xb = r;
            // the block's radius range and hi residual (lane b & 63 of the item's registers)
            const int bi = cc.blk;
            const float b_lo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bi < 64 ? bl_lo[0] : bl_lo[1]), bi & 63));
            const float b_hi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bi < 64 ? bl_hi[0] : bl_hi[1]), bi & 63));
            const float b_re = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bi < 64 ? bl_re[0] : bl_re[1]), bi & 63));
            refresh(b_lo, b_hi, b_re);
            tick(4);
#pragma unroll
            for (int cg = 0; cg < 4; ++cg) acc[cg] = (wf32x16)(0.0f);
            if (cnt && lane == 0) {
                if (wave == 0) atomicAdd(cnt + 2, 1ull);
                if (!wdead) atomicAdd(cnt + 0, 32ull * 128ull);
            }
        }
        if (!wdead) {
            if (j == 0) mfma_slot(std::integral_constant<int, 0>{}, r);
            if (NSL > 1 && j == 1) mfma_slot(std::integral_constant<int, (NSL > 1 ? 1 : 0)>{}, r);
            if (NSL > 2 && j == 2) mfma_slot(std::integral_constant<int, (NSL > 2 ? 2 : 0)>{}, r);
            if (NSL > 3 && j == 3) mfma_slot(std::integral_constant<int, (NSL > 3 ? 3 : 0)>{}, r);
            if (kWClk) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            tick(5);
            if (j == NSL - 1) select();
            tick(6);
        }
        advance(cc);
    }
    if (kWClk && a.stats && lane == 0 && (wave == 0 || wave == SW)) {
        // wave 0: [0] loop total, [1] DMA wait + barrier, [2] DMA issue, [3] item transitions,
        // [4] refresh, [5] MFMA (issue), [6] selection; wave SW: [7] item claims
        if (wave == 0) {
            atomicAdd(a.stats + 0, (unsigned long long)(clock64() - t0));
            for (int i = 1; i < 7; ++i) atomicAdd(a.stats + i, (unsigned long long)ck[i]);
        } else {
            atomicAdd(a.stats + 7, (unsigned long long)ck[7]);
        }
    }
}

// ------------------------------------------------------------------ host side
template <int NKS>
static hipError_t launch_w(const WArgs &a, int grid, hipStream_t st) {
    static std::atomic<uint64_t> attr{0};
    hipError_t e = set_smem_attr_once(attr, (const void *)k_screen_w<NKS>, WSmem::total);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_screen_w<NKS>), dim3(grid), dim3(512), WSmem::total, st, a);
    return hipGetLastError();
}

bool wscreen_shape_ok(int64_t dpad) { return dpad == 64 || dpad == 96 || dpad == 128; }
int wscreen_smem() { return WSmem::total; }

hipError_t launch_pairs(const float *Q, int64_t d, const int32_t *probe, int64_t npairs, int nprobe, int n_lists,
                        const float *pivot, int centred, const float2 *lstat, const uint32_t *qbound,
                        int32_t *probe_live, float4 *QN, float *QE, float *pqn, uint16_t *QH, int64_t dpad,
                        hipStream_t st) {
    const unsigned g = (unsigned)((npairs * 16 + 255) / 256);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pairs, dim3(g), dim3(256), 0, st, Q, d, probe, npairs, nprobe, n_lists, pivot, centred, lstat,
                       qbound, probe_live, QN, QE, pqn, QH, dpad);
    return hipGetLastError();
}

hipError_t launch_wscreen(const lira_index *idx, const float *q, const int32_t *cnt, const int32_t *qoff,
                          const int32_t *qlist, const int4 *itab, int32_t *head, const float4 *QN, const float *QE,
                          u64 *partial, float *pE, uint32_t *qbound, int nprobe, int k, int bpc, int bpc_near,
                          int nch_max, int n_virt, int tri, int grid, int4 *wrec, int64_t max_items, hipStream_t st) {
    // per-item records (the plan's item count is on the device: one thread per possible item)
    hipLaunchKernelGGL(k_wrec, dim3((unsigned)((max_items + 255) / 256)), dim3(256), 0, st, itab, head, idx->tile_off,
                       qoff, cnt, idx->rmaxc, (int)idx->n_lists, n_virt, bpc, bpc_near, wrec);
    WArgs a;
    a.wrec = wrec;
    a.Xb = idx->Xb;
    a.xadj = idx->xadjc;
    a.rmax = idx->rmaxc;
    a.tile_off = idx->tile_off;
    a.cnt = cnt;
    a.qoff = qoff;
    a.qlist = qlist;
    a.itab = itab;
    a.head = head;
    a.Q = q;
    a.pivot = idx->pivot;
    a.QN = QN;
    a.QE = QE;
    a.tstat = tri ? idx->tstat : nullptr;
    a.tres = idx->tres;
    a.partial = partial;
    a.pE = pE;
    a.qbound = qbound;
    a.d = idx->d;
    a.dpad = idx->dpad;
    a.n_lists = (int)idx->n_lists;
    a.n_virt = n_virt;
    a.nprobe = nprobe;
    a.k = k;
    a.bpc = bpc;
    a.bpc_near = bpc_near;
    a.nch_max = nch_max;
    a.share = idx->opt.share;
    a.tri = tri && idx->tstat != nullptr;
    a.stats = idx->stats_on ? (unsigned long long *)idx->stats : nullptr;
    switch (idx->dpad) {
        case 64: return launch_w<4>(a, grid, st);
        case 96: return launch_w<6>(a, grid, st);
        case 128: return launch_w<8>(a, grid, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace lira
