// lira_screen.hip -- screened candidate scan with exact re-check (gfx950).
// Default path of lira_scan_topk; replaces search.cpp:468-514 and the
// per-(query, bucket) faiss IndexFlat*.search calls (LIRA_smallscale.py:158-172)
// with results identical to the all-exact scan (lira_scan.hip k_scan).
//
// Why.  search.cpp's distance is a sequential fp32 sum of separately rounded
// terms: fl(fl(q-x)^2) for L2 (3 VALU ops per candidate-dim, no FMA allowed)
// and fl(q*x) for IP (2 ops).  Computing that for every candidate makes the
// scan VALU-bound at 3 ops/dim.  Here every candidate is first *screened* with
// a dot product on the matrix cores -- by default bf16 parts of the (L2:
// pivot-centred) vectors on v_mfma_f32_16x16x32_bf16 (k_screen_m, SPLIT 1-3;
// the fp32 forms: v_mfma_f32_16x16x4_f32, or v_pk_fma_f32 in k_screen) -- and
// only the few candidates that can still reach the top-k are re-computed in the
// reference's arithmetic (k_smerge).  Nothing is approximated: the screen is a
// rigorous filter, so the output is bit-identical.  The error model below is
// the fp32 screen's; err_E carries the split forms' terms.
//
// Error model (u = 2^-24, per (query, partition); double on the host side of
// each bound, fp32 values rounded in the safe direction):
//   L2:  s~ = fma(-2, dot, fl(qn + xn)) with qn = fl(||q||^2), xn = fl(||x||^2)
//        and dot an fp32 FMA chain, so |s~ - D| <= E = 1.05 (d+8) u (|q|+R)^2 + dl,
//        D = ||q-x||^2 real, R >= max ||x|| of the partition, dl = d 2^-140
//        (underflow).  search.cpp's sum s (all terms >= 0) satisfies
//        D (1-g) - dl <= s <= D (1+g) + dl with g = (d+4) u.
//   IP:  score = -ip; |s - (-dot)| <= E = 1.05 * 2 (d+2) u |q| R + dl.
// A list's k-th screened score s~k therefore bounds the final k-th exact score
// by P = (s~k + E)(1+g) + dl (IP: s~k + E), and a candidate can only matter if
// its s~ <= lim(T) = (T + dl)/(1-g) + E (IP: T + E), T = the best such bound
// known.  The per-block test is that inequality on the dot product with one
// more rounding absorbed (see row_h).
//
// Schedule: as k_scan (partition-major items of QR queries x a chunk of the
// bucket, persistent grid, atomic work head).  X tiles stream through a 2-deep
// LDS ring by LDS-DMA; each wave owns RW = QR/4 query rows and all 256
// candidates of a block (4 per lane); the rows' query values come from a
// per-item transposed copy (k_qstage) through scalar loads, so the inner step
// is one ds_read_b128 + RW*2 v_pk_fma_f32 with SGPR-broadcast operands.
//
// Selection per row: a sorted list of K2 = 32*RL >= k+8 screened keys
// (s~ << 32 | storage row) in LDS with a 32-key survivor buffer (ballot
// compaction, half-wave bitonic merge when full).  k_smerge then takes, per
// query, every listed candidate with s~ <= lim(T_final), re-computes its exact
// score from the tiles, and selects/dedups exactly as k_merge.  A list whose
// K2-th key is still inside lim may have dropped a needed candidate: k_smerge
// then re-scans that chunk exactly (never seen in the benches; tested).
#include <algorithm>
#include <cstdlib>
#include <string>

#include "lira_bounds.hpp"
#include "lira_device.hpp"
#include "lira_internal.hpp"
#include "lira_rscreen.hpp"

#include <cmath>

namespace lira {

hipError_t launch_plan(const lira_index *idx, const int32_t *probe, int64_t npairs, int nprobe, int bpc,
                       int bpc_near,
                       int qr, int groups, int32_t *cnt, int32_t *cursor, int32_t *qoff, int32_t *item_off,
                       int32_t *nch, int32_t *head, int32_t *qlist, int32_t *qblk_off, int4 *itab,
                       hipStream_t st, int bpc_near_min, int workers, int near_div, int near0,
                       const int32_t *cnt8 = nullptr);

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) float cfloat;  // uniform address -> s_load

static constexpr int kSBT = 4;     // tiles per candidate block (256 candidates)
static constexpr int kSDK = 16;    // dims per staged chunk
static constexpr int kSThreads = 256;

struct ScreenArgs {
    const float *X;        // [n_tiles][dpad][64]
    const float *xadj;     // [n_tiles*64]
    const float *rmax;     // [n_lists]
    const int32_t *tile_off, *cnt, *item_off, *qblk_off;
    const int4 *itab;  // item -> (virtual partition, query block, chunk, global query block)
    // per-pair query records (k_screen_m<..., 3>, qpair = 1): a row's pair is
    // qlist[qoff[vp] + qb QR + row], its QN / QE are indexed by pair, and its hi
    // parts are gathered from QH[pair][dpad] (no k_qstage copy)
    const int32_t *qoff, *qlist;
    const uint16_t *QH;
    int qpair;
    int32_t *head;
    const float *QT;       // [qblk][dpad][QR]
    const float4 *QN;      // [qblk*QR]: qn, |q| (up), pair (int bits), 0
    const float *QE;       // [qblk*QR]: ||q - hi(q)|| (up) of the staged row (SPLIT 3)
    u64 *partial;          // [pair][nch_max][K2]
    float *pE;             // [pair][nch_max]: k_screen_m's bound on its listed keys' screening error
    uint32_t *qbound;      // [nq] f2ord(bound on the final k-th exact score); NULL = off
    int64_t d, dpad;
    int n_lists, n_virt, nprobe, k, bpc, nch_max;  // n_virt = groups * n_lists (virtual partitions)
    int bpc_near;  // blocks per chunk of group 0 (each query's nearest partition) when n_virt > n_lists
    unsigned long long *stats;  // NULL or lira_index_set_stats counters
    // L2 triangle-inequality block skip (k_screen_m): queries, per-list pivot,
    // per-tile radius bounds (lira_abi.hip k_pivot_final / k_row_stats); NULL = off
    const float *Q;
    const float *pivot;
    const float2 *tstat;
    const float *tres;  // per tile max ||x - hi(x)|| of the split copy (NULL: 2^-8 R bounds it)
    int share;     // k_screen_m: publish/re-read the query bound every block (else once per item)
    int split;     // k_screen_m<..., SPLIT = 1>: X is the split-bf16 copy (Xb), QT in the split layout
    int centred;   // (L2, split) Xb / QT hold x - c / q - c of the list's pivot; xadj, rmax, QN are theirs
    int dbg;  // timing experiments only (LIRA_OPT_DEBUG, -DLIRA_DEBUG builds; results invalid): 1 = no MFMA, 2 = no selection,
             // 4 = no X/Q staging, 8 = per-phase clocks into stats 1/3/6 (k_screen_m)
};

// ---- Q staging: transposed per-item query copy + norms ---------------------
// Block b = one query block (virtual partition v, block qb of QR pairs).
// QN.w = fl(||q - pivot_p||) (double sum, round to nearest: the true value is
// within 1 ulp) for the triangle skip, when a pivot array is given.
// SPLIT: QT per query block and 16-dim chunk c is [g 4][QR rows][8 bf16]
// (64 QR bytes, the fp32 chunk's size), g = 2 hl + h holding the hi/lo part
// of dims 16c + 8h .. +7 of the row: the A fragments of k_screen_m<SPLIT>.
//
// cpivot (L2, split): centre the rows on their partition's pivot, fl(q - c),
// before splitting; QN.x / QN.y are then the centred norms, and pqn[pair] =
// QN.y (the merge's copy of the row's norm).
// Last v in [0, n) with off[v] <= b (off nondecreasing, off[0] <= b), by one
// whole wave: a 64-ary search, ceil(log64 n) dependent rounds of loads instead
// of log2 n (k_qstage's thread-0 binary search was ~7 dependent global loads
// per workgroup).  Wave-uniform result.
__device__ __forceinline__ int wave_find_owner(const int32_t *off, int n, int b) {
    const int lane = threadIdx.x & 63;
    int lo = 0;
    while (n > 1) {
        const int stride = (n + 63) / 64, o = lane * stride;
        const bool ok = o < n && off[lo + o] <= b;
        const int L = __popcll(__ballot(ok));  // lanes 0 .. L-1 (monotone; lane 0 always)
        lo += (L - 1) * stride;
        n = min(stride, n - (L - 1) * stride);
    }
    return lo;
}

static constexpr int kQSlabs = 1;  // 64-dim slabs per k_qstage workgroup
template <int QR, bool SPLIT>
__global__ __launch_bounds__(256) void k_qstage(const float *Q, int64_t d, int64_t dpad, int nprobe,
                                                int n_virt, int n_lists, const int32_t *cnt, const int32_t *qoff,
                                                const int32_t *qlist, const int32_t *qblk_off, const float *pivot,
                                                const float *cpivot, float *QT, float4 *QN, float *pqn,
                                                float *QE) {
    __shared__ int pairs[QR], qrow_s[QR];
    __shared__ int s_v;
    __shared__ float tr[64][65];
    const int b = blockIdx.x;
    if (b >= qblk_off[n_virt]) return;
    if (threadIdx.x < 64) {
        const int v = wave_find_owner(qblk_off, n_virt, b);
        if (threadIdx.x == 0) s_v = v;
    }
    __syncthreads();
    const int v = s_v, qb = b - qblk_off[v];
    const int nval = min(QR, cnt[v] - qb * QR);
    const float *cpv = cpivot ? cpivot + (int64_t)(v >= n_lists ? v - n_lists : v) * d : nullptr;
    if (threadIdx.x < QR) {
        const int pr = (int)threadIdx.x < nval ? qlist[qoff[v] + qb * QR + threadIdx.x] : -1;
        pairs[threadIdx.x] = pr;
        qrow_s[threadIdx.x] = pr >= 0 ? pr / nprobe : -1;
    }
    __syncthreads();
    // transpose through LDS, 64 rows x 64 dims at a time: reads along the
    // query row, writes along QT's row axis, both coalesced
    constexpr int RT = QR < 64 ? QR : 64;  // rows per transpose tile
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // blockIdx.y: this workgroup's group of kQSlabs 64-dim slabs (many
    // workgroups per query block: GIST1M plan 0.38 -> 0.23 ms, SIFT1M 0.17 -> 0.15)
    const int64_t j_lo = (int64_t)blockIdx.y * kQSlabs * 64, j_hi = min<int64_t>(dpad, j_lo + kQSlabs * 64);
    for (int r0 = 0; r0 < QR; r0 += RT) {
        for (int64_t j0 = j_lo; j0 < j_hi; j0 += 64) {
            const int64_t j = j0 + lane;
            // the wave's RT/4 rows: every load issued before the first store
            constexpr int PER = RT / 4;
            float qv[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int qi = qrow_s[r0 + wv + 4 * i];
                qv[i] = qi >= 0 && j < d ? Q[(int64_t)qi * d + j] : 0.0f;
            }
            const float cv = cpv && j < d ? cpv[j] : 0.0f;
#pragma unroll
            for (int i = 0; i < PER; ++i) tr[wv + 4 * i][lane] = cpv && j < d ? qv[i] - cv : qv[i];
            __syncthreads();
            if (SPLIT) {
                // units (chunk cc of the slab, g, row): 16 B each, rows fastest
                for (int u = threadIdx.x; u < 16 * RT; u += 256) {
                    const int row = u % RT, cg = u / RT, cc = cg >> 2, gg = cg & 3;
                    const int64_t c0 = j0 + 16 * cc;
                    if (c0 >= dpad || (QE && gg >= 2)) continue;  // (hi x hi: lo parts unused)
                    uint32_t wd[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = 16 * cc + 8 * (gg & 1) + 2 * e;
                        wd[e] = bf16_split_part(tr[row][j], gg >> 1) | (bf16_split_part(tr[row][j + 1], gg >> 1) << 16);
                    }
                    ((uint4 *)QT)[((int64_t)b * dpad + c0) * QR / 4 + (int64_t)gg * QR + r0 + row] =
                        make_uint4(wd[0], wd[1], wd[2], wd[3]);
                }
            } else if (lane < RT) {
                for (int jj = wv; jj < 64 && j0 + jj < dpad; jj += 4)
                    QT[((int64_t)b * dpad + j0 + jj) * QR + r0 + lane] = tr[lane][jj];
            }
            __syncthreads();
        }
    }
    // the rows' norms, spread over the slab groups (each row whole in one);
    // four rows per wave at a time, so their loads are in flight together
    const float *pv = pivot ? pivot + (int64_t)(v >= n_lists ? v - n_lists : v) * d : nullptr;
    constexpr int NM = 4;  // rows per wave at a time (8: GIST1M plan 0.16 -> 0.21 ms)
    const int rstep = 4 * gridDim.y;
    for (int r0 = blockIdx.y + gridDim.y * wv; r0 < QR; r0 += NM * rstep) {
        int qi[NM];
        double s[NM], t[NM], e[NM];  // e: the hi parts' residual (QE)
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const int r = r0 + m * rstep;
            qi[m] = r < QR ? qrow_s[r] : -1;
            s[m] = t[m] = e[m] = 0.0;
        }
        for (int64_t j = lane; j < d; j += 64) {
            const float cv = cpv ? cpv[j] : 0.0f, pj = pv ? pv[j] : 0.0f;
            float xv[NM];
#pragma unroll
            for (int m = 0; m < NM; ++m) xv[m] = qi[m] >= 0 ? Q[(int64_t)qi[m] * d + j] : 0.0f;
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                if (qi[m] < 0) continue;  // (no pair: zero norms)
                const double x = (double)xv[m];
                const float sv = cpv ? xv[m] - cv : xv[m];  // the staged value
                const double xc = (double)sv;
                s[m] = __builtin_fma(xc, xc, s[m]);
                if (SPLIT && QE) {  // sv - hi(sv): exact in fp32
                    const double rr = (double)(sv - __uint_as_float(bf16_rne_sat(sv) << 16));
                    e[m] = __builtin_fma(rr, rr, e[m]);
                }
                if (pv) {
                    const double df = x - (double)pj;
                    t[m] = __builtin_fma(df, df, t[m]);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < NM; ++m) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {  // (DPP / swizzle exchanges, lira_device.hpp)
                s[m] += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, s[m]), o));
                if (pivot) t[m] += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, t[m]), o));
                if (SPLIT && QE) e[m] += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, e[m]), o));
            }
        }
        if (lane < NM) {  // lane m writes row r0 + m * rstep
            double sm = s[0], tm = t[0], em = e[0];
#pragma unroll
            for (int m = 1; m < NM; ++m)
                if (lane == m) {
                    sm = s[m];
                    tm = t[m];
                    em = e[m];
                }
            const int r = r0 + lane * rstep;
            if (r < QR) {
                const int pr = pairs[r];
                const float qnu = __double2float_ru(__builtin_sqrt(sm) * (1.0 + 0x1p-40));
                QN[(int64_t)b * QR + r] = make_float4((float)sm, qnu, __int_as_float(pr), (float)__builtin_sqrt(tm));
                if (pqn && pr >= 0) pqn[pr] = qnu;
                if (SPLIT && QE) QE[(int64_t)b * QR + r] = __double2float_ru(__builtin_sqrt(em) * (1.0 + 0x1p-40));
            }
        }
    }
}

// ---- the screening kernel --------------------------------------------------
// MF: the k_screen_m carve (xadj stage, block ranges); XH: hi-only x
// (k_screen_m<..., SPLIT = 2>): half the X bytes per chunk and a 3-deep ring
// HH: the hi x hi screen (k_screen_m<..., SPLIT = 3>): a slot holds 32 dims, the
// hi parts of x (4 KiB per tile) and of the queries (QR * 64 B), 2 slots
template <int QR, int RL, bool MF = false, bool XH = false, bool HH = false>
struct SSmem {
    static constexpr int RW = QR / 4, K2 = 32 * RL, BC = 32;
    static constexpr int kXT = (XH ? 2 : 4) * 1024;         // one tile's chunk (XH: the hi parts; HH: 32 dims of them)
    static constexpr int kXS = kSBT * kXT;                  // X chunk: 16 KiB (XH: 8)
    static constexpr int kQS = kSDK * QR * 4;               // Q chunk: 4 KiB at QR = 64 (HH: 32 dims of hi parts)
    static constexpr int kXA = 0;                           // (k_screen: none)
    static constexpr int kStage = kXS + kQS + kXA;
    static constexpr int NSL = XH && !HH ? 3 : 2;           // ring slots
    // (MF) the xadj of the last two blocks, [2][256] (staged with a block's first chunk)
    static constexpr int kXB = MF ? 2 * kSBT * kTile * 4 : 0;
    static constexpr int kX = NSL * kStage + kXB;
    static constexpr int kLists = QR * K2 * 8;
    static constexpr int kBufs = QR * BC * 8;
    // item; pair, bufc, (spare) per row; block-skip (A, B) x 2 parities and
    // ||q - pivot|| (lo, hi) doubles per row; (MF) the radius range of each of
    // an item's first kBR blocks
    static constexpr int kBR = MF ? 128 : 0;
    static constexpr int kMeta = 64 + QR * 4 * 3 + 2 * QR * 8 + QR * 16 + kBR * 8 + (XH || HH ? kBR * 4 : 0);
    static constexpr int total = kX + kLists + kBufs + kMeta;
};

typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ void sglds16(const void *gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_addr)
        : "memory");
}

// The same DMA through the compiler builtin (hipcc sets M0 itself and counts
// the load in its own vmcnt bookkeeping)
__device__ __forceinline__ void sglds16b(const void *gsrc, uint32_t lds_addr) {
    __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void *)(uintptr_t)lds_addr, 16, 0, 0);
}

#ifdef LIRA_PHASE_CLOCKS
static constexpr bool kPhaseClocks = true;
#else
static constexpr bool kPhaseClocks = false;
#endif
#if defined(LIRA_DEBUG) || defined(LIRA_PHASE_CLOCKS)
bool debug_build() { return true; }
#else
bool debug_build() { return false; }
#endif
#ifndef LIRA_SGLDS
#define LIRA_SGLDS sglds16
#endif

// acc += x * splat(q.lo) / splat(q.hi) on packed fp32.  Inline asm: hipcc
// otherwise copies every odd-register splat source with a v_mov first (one
// extra VALU op per 8 FMAs), while op_sel reads either half in place.
__device__ __forceinline__ void pkfma_lo(f2 &acc, f2 x, f2 q) {
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(x), "v"(q));
}
__device__ __forceinline__ void pkfma_hi(f2 &acc, f2 x, f2 q) {
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(x), "v"(q));
}

// the value lane 4 g + reg holds (lanes 0..15: one per query row), for every
// lane of group g (4 v_readlane instead of a ds_bpermute)
__device__ __forceinline__ float from_row_lane(float v, int reg, int g) {
    const float a0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), reg));
    const float a1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 4 + reg));
    const float a2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 8 + reg));
    const float a3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 12 + reg));
    return g == 0 ? a0 : g == 1 ? a1 : g == 2 ? a2 : a3;
}


// Merge a row's survivor buffer (n keys) into its sorted K2-list.  Both halves
// run the half-wave network on the same row; half 0 stores.
template <int RL>
__device__ __forceinline__ void s_flush(u64 *L, const u64 *buf, int n) {
    const int hl = lane_id() & 31;
    u64 lst[RL];
#pragma unroll
    for (int r = 0; r < RL; ++r) lst[r] = L[r * 32 + hl];
    const u64 b = hl < n ? buf[hl] : kEmptyKey;
    half_merge_batch1<RL>(lst, b);
    if (lane_id() < 32) {
#pragma unroll
        for (int r = 0; r < RL; ++r) L[r * 32 + hl] = lst[r];
    }
    __builtin_amdgcn_wave_barrier();
}

// Two rows at once: half 0 merges buffer A (na keys) into list A, half 1
// buffer B into list B (the half-wave network sorts both halves independently).
template <int RL>
__device__ __forceinline__ void s_flush2(u64 *LA, const u64 *bufA, int na, u64 *LB, const u64 *bufB, int nb) {
    const int hl = lane_id() & 31;
    const bool hi = lane_id() >= 32;
    u64 *L = hi ? LB : LA;
    const u64 *buf = hi ? bufB : bufA;
    const int n = hi ? nb : na;
    u64 lst[RL];
#pragma unroll
    for (int r = 0; r < RL; ++r) lst[r] = L[r * 32 + hl];
    const u64 b = hl < n ? buf[hl] : kEmptyKey;
    half_merge_batch1<RL>(lst, b);
#pragma unroll
    for (int r = 0; r < RL; ++r) L[r * 32 + hl] = lst[r];
    __builtin_amdgcn_wave_barrier();
}

// Append this lane's passing keys (v-major order) to the row's buffer,
// merging into the list whenever the buffer fills.  Returns the new fill.
template <int RL>
__device__ __forceinline__ int s_append(u64 *L, u64 *buf, int bc, u64 k0, u64 k1, u64 k2, u64 k3, int pmask,
                                     unsigned long long *stats) {
    const u64 key[4] = {k0, k1, k2, k3};
    u64 b[4];
    int pos[4], tot = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        b[v] = __ballot((pmask >> v) & 1);
        pos[v] = tot + mbcnt64(b[v]);
        tot += popc64(b[v]);
    }
    if (stats && lane_id() == 0) atomicAdd(stats + 7, (unsigned long long)tot);
    int consumed = 0;
    for (;;) {
        const int room = 32 - bc;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int rel = pos[v] - consumed;
            if (((pmask >> v) & 1) && rel >= 0 && rel < room) buf[bc + rel] = key[v];
        }
        const int placed = min(room, tot - consumed);
        bc += placed;
        consumed += placed;
        __builtin_amdgcn_wave_barrier();
        if (bc == 32) {
            s_flush<RL>(L, buf, 32);
            bc = 0;
        }
        if (consumed >= tot) break;
    }
    return bc;
}

// s_append for NV keys per lane (v-major order), bit v of pmask = key v passes.
template <int RL, int NV>
__device__ __forceinline__ int s_append_n(u64 *L, u64 *buf, int bc, const u64 (&key)[NV], int pmask,
                                          unsigned long long *stats) {
    u64 b[NV];
    int pos[NV], tot = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        b[v] = __ballot((pmask >> v) & 1);
        pos[v] = tot + mbcnt64(b[v]);
        tot += popc64(b[v]);
    }
    if (stats && lane_id() == 0) atomicAdd(stats + 7, (unsigned long long)tot);
    int consumed = 0;
    for (;;) {
        const int room = 32 - bc;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int rel = pos[v] - consumed;
            if (((pmask >> v) & 1) && rel >= 0 && rel < room) buf[bc + rel] = key[v];
        }
        const int placed = min(room, tot - consumed);
        bc += placed;
        consumed += placed;
        __builtin_amdgcn_wave_barrier();
        if (bc == 32) {
            s_flush<RL>(L, buf, 32);
            bc = 0;
        }
        if (consumed >= tot) break;
    }
    return bc;
}

template <int METRIC, int RL, int QR, int OCC>
__global__ __launch_bounds__(kSThreads, OCC) void k_screen(ScreenArgs a) {
    typedef SSmem<QR, RL> S;
    constexpr int RW = S::RW, K2 = S::K2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *Xs = (float *)smem;  // [2] x {X: [4 tiles][16 dims][64], Q: [16 dims][QR]}
    u64 *lists = (u64 *)(smem + S::kX);                      // [QR][K2]
    u64 *bufs = (u64 *)(smem + S::kX + S::kLists);           // [QR][32]
    int *meta = (int *)(smem + S::kX + S::kLists + S::kBufs);
    int *m_pair = meta + 16, *m_bufc = meta + 16 + QR;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int k = a.k;
    const double dd = (double)a.d;
    const float4 *Xg = (const float4 *)a.X;
    const uint32_t xs_lds = (uint32_t)(uintptr_t)(lds_void_t *)Xs;
    const int tstride = (int)a.dpad * (kTile / 4);  // float4 per tile
    const int nchunk = (int)(a.dpad / kSDK);
    const int ti = lane >> 4, col = (lane & 15) * 4;   // this lane's 4 candidates of a block

    __shared__ int xq[9];  // the XCD queues' bounds (k_plan)
    int qx = 0, qtries = 0, nxt = -1;  // thread 0: its queue, the claimed next item
    if (tid == 0) {
        for (int r = 0; r < 9; ++r) xq[r] = a.head[10 + r];
        qx = xcd_id();
        nxt = claim_item(a.head, xq, qx, qtries);
    }  // thread 0: the claimed next item
    for (;;) {
        if (tid == 0) {
            // the next item is claimed one item ahead (its atomic completes
            // under this item's work); one table load decodes it
            const int item = nxt;
            const int ok = item >= 0;
            int4 e = make_int4(0, 0, 0, 0);
            if (ok) {
                e = a.itab[item];
                nxt = claim_item(a.head, xq, qx, qtries);
            }
            meta[0] = ok;
            meta[1] = e.x;
            meta[2] = e.y;
            meta[3] = e.z;
            meta[4] = e.w;
        }
        __syncthreads();
        if (!meta[0]) break;
        const int vp = __builtin_amdgcn_readfirstlane(meta[1]);  // virtual partition
        const int p = vp >= a.n_lists ? vp - a.n_lists : vp;
        const int ch = __builtin_amdgcn_readfirstlane(meta[3]);
        const int gqb = __builtin_amdgcn_readfirstlane(meta[4]);
        if (tid < QR) {
            m_pair[tid] = __float_as_int(a.QN[(int64_t)gqb * QR + tid].z);
            m_bufc[tid] = 0;
        }
        for (int i = tid; i < QR * K2; i += kSThreads) lists[i] = kEmptyKey;
        __syncthreads();

        const int tile0 = __builtin_amdgcn_readfirstlane(a.tile_off[p]);
        const int ntl = __builtin_amdgcn_readfirstlane(a.tile_off[p + 1]) - tile0;
        const int bpc = vp < a.n_lists && a.n_virt > a.n_lists ? a.bpc_near : a.bpc;
        const int tb_begin = ch * bpc * kSBT;
        const int tb_end = min(ntl, tb_begin + bpc * kSBT);
        const double R = (double)a.rmax[p];

        // this lane's row for threshold work: row = wave*RW + (lane % RW)
        const int my_row = wave * RW + (lane % RW);
        const float4 qrec = a.QN[(int64_t)gqb * QR + my_row];
        const int my_pair = __float_as_int(qrec.z);
        const int my_q = my_pair >= 0 ? my_pair / a.nprobe : -1;
        const double my_qn = (double)qrec.x, my_qnorm = (double)qrec.y;
        const double my_E = err_E<METRIC>(my_qnorm, R, dd);
        u64 *my_list = lists + my_row * K2;

        const float4 *qtg = (const float4 *)(a.QT + (int64_t)gqb * a.dpad * QR);

        // Stage chunk (tb, jc) into ring slot `slot` by LDS-DMA: wave w moves
        // 1 KiB of each of the block's 4 tile chunks (tiles past the block's
        // end re-read its last valid one; masked by xadj = +inf) and, for
        // w < QR/16, 1 KiB of the Q chunk
        auto stage = [&](int tb, int jc, int slot) {
            const int ntv = min(kSBT, tb_end - tb);
            const float4 *src = Xg + (int64_t)(tile0 + tb) * tstride + jc * (kTile / 4) + tid;
            const uint32_t base = xs_lds + (uint32_t)(slot * S::kStage);
            const uint32_t dst = __builtin_amdgcn_readfirstlane(base + (uint32_t)(wave * 256) * 4u);
#pragma unroll
            for (int i = 0; i < kSBT; ++i)
                sglds16(src + min(i, ntv - 1) * tstride, dst + (uint32_t)(i * (kSDK * kTile) * 4));
            if (wave < QR / 16)
                sglds16(qtg + (int64_t)jc * (QR / 4) + wave * 64 + lane,
                        __builtin_amdgcn_readfirstlane(base + (uint32_t)S::kXS + (uint32_t)wave * 1024u));
        };
        int slot = 0;
        if (tb_begin < tb_end) stage(tb_begin, 0, 0);

#pragma unroll 1
        for (int tb = tb_begin; tb < tb_end; tb += kSBT) {
            const int ntv = min(kSBT, tb_end - tb);
            // screening constants of my 4 candidates (+inf: padding / past the block)
            f4 a4 = (f4)(__builtin_inff());
            if (ti < ntv) a4 = *(const f4 *)&a.xadj[(int64_t)(tile0 + tb + ti) * kTile + col];
            const uint32_t pub = a.qbound && my_q >= 0
                ? __hip_atomic_load(a.qbound + my_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;

            f2 acc[RW][2];
#pragma unroll
            for (int r = 0; r < RW; ++r) acc[r][0] = acc[r][1] = (f2)(0.0f);

#pragma unroll 1
            for (int c = 0; c < nchunk; ++c) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA landed
                __syncthreads();  // every wave's DMA landed; every wave is done with the other slot
                {
                    int njc = (c + 1) * kSDK, ntb = tb;
                    if (c + 1 == nchunk) {
                        njc = 0;
                        ntb = tb + kSBT;
                    }
                    if (ntb < tb_end) stage(ntb, njc, slot ^ 1);
                }
                const float *sb = (const float *)((const char *)Xs + slot * S::kStage);
                const float *xp = sb + ti * (kSDK * kTile) + col;
                const float *qp = sb + S::kXS / 4 + wave * RW;  // this wave's rows; broadcast reads
#pragma unroll
                for (int j = 0; j < kSDK; ++j) {
                    const f4 x = *(const f4 *)(xp + j * kTile);
                    const f2 xa = x.xy, xb = x.zw;
#pragma unroll
                    for (int r4 = 0; r4 < RW / 4; ++r4) {
                        const f4 q4 = *(const f4 *)(qp + j * QR + r4 * 4);
                        const f2 q01 = q4.xy, q23 = q4.zw;
                        pkfma_lo(acc[r4 * 4 + 0][0], xa, q01);
                        pkfma_lo(acc[r4 * 4 + 0][1], xb, q01);
                        pkfma_hi(acc[r4 * 4 + 1][0], xa, q01);
                        pkfma_hi(acc[r4 * 4 + 1][1], xb, q01);
                        pkfma_lo(acc[r4 * 4 + 2][0], xa, q23);
                        pkfma_lo(acc[r4 * 4 + 2][1], xb, q23);
                        pkfma_hi(acc[r4 * 4 + 3][0], xa, q23);
                        pkfma_hi(acc[r4 * 4 + 3][1], xb, q23);
                    }
                }
                slot ^= 1;
            }

            // ---- thresholds: lane (row) computes h from its list and the published bound
            float h_l;
            {
                const u64 kk = my_list[k - 1];
                double T = kk == kEmptyKey ? __builtin_inf() : bound_P<METRIC>((double)key_score(kk), my_E, dd);
                if (pub != ~0u) T = fmin(T, (double)ord2f(pub));
                h_l = my_pair < 0 ? __builtin_inff()  // no query: nothing passes
                                  : row_h<METRIC>(s_lim<METRIC>(T, my_E, dd), my_qn, my_qnorm, R);
            }
            if (a.stats && lane == 0) {
                if (wave == 0) atomicAdd(a.stats + 2, 1ull);
                atomicAdd(a.stats + 0, (unsigned long long)RW * kSBT * kTile);  // (row, candidate) pairs screened
            }

            // ---- selection.  Phase 1 (unrolled): per row, which of my 4
            // candidates pass h; rows where any lane has one set `hit`
            // (wave-uniform).  Phase 2 (one copy of the code): those rows.
            int vmask = 0;  // real candidates (padding has xadj = +inf)
            vmask |= a4.x != __builtin_inff() ? 1 : 0;
            vmask |= a4.y != __builtin_inff() ? 2 : 0;
            vmask |= a4.z != __builtin_inff() ? 4 : 0;
            vmask |= a4.w != __builtin_inff() ? 8 : 0;
            uint32_t hit = 0;
            u64 pmw = 0;
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                const float h = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h_l), r));
                const f2 w0 = acc[r][0] - a4.xy, w1 = acc[r][1] - a4.zw;
                const int pm = ((w0.x >= h) | ((w0.y >= h) << 1) | ((w1.x >= h) << 2) | ((w1.y >= h) << 3)) & vmask;
                pmw |= (u64)pm << (4 * r);
                if (__any(pm)) hit |= 1u << r;
            }
            hit = __builtin_amdgcn_readfirstlane(hit);
            while (hit) {
                const int r = __builtin_ctz(hit);
                hit &= hit - 1;
                const int row = wave * RW + r;
                // this row's dot products (uniform r: a select chain, no
                // dynamic register indexing)
                f2 d0 = acc[0][0], d1 = acc[0][1];
#pragma unroll
                for (int rr = 1; rr < RW; ++rr) {
                    d0 = r == rr ? acc[rr][0] : d0;
                    d1 = r == rr ? acc[rr][1] : d1;
                }
                float h = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h_l), r));
                int pm = (int)(pmw >> (4 * r)) & 15;
                const float qnf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int((float)my_qn), r));
                const float av[4] = {a4.x, a4.y, a4.z, a4.w};
                const float dv[4] = {d0.x, d0.y, d1.x, d1.y};
                float sc[4];  // screened scores (+inf for padding)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    if (METRIC == LIRA_METRIC_L2)
                        sc[v] = (vmask >> v) & 1 ? __builtin_fmaf(-2.0f, dv[v], qnf + 2.0f * av[v]) : __builtin_inff();
                    else
                        sc[v] = (vmask >> v) & 1 ? -dv[v] : __builtin_inff();
                }
                if (h == -__builtin_inff()) {
                    // no bound yet (an item's first block): take one from the
                    // block itself.  t = ceil(k/64) smallest per lane, j =
                    // ceil(k/t): the j-th smallest lane value has >= j*t >= k
                    // real candidates at or below it.
                    float srt[4] = {sc[0], sc[1], sc[2], sc[3]};
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int v = 0; v + 1 < 4 - i; ++v) {
                            const float lo = fminf(srt[v], srt[v + 1]), hi = fmaxf(srt[v], srt[v + 1]);
                            srt[v] = lo;
                            srt[v + 1] = hi;
                        }
                    const int t = (k + 63) / 64;
                    const float mine = t <= 1 ? srt[0] : t == 2 ? srt[1] : t == 3 ? srt[2] : srt[3];
                    const uint32_t sorted = wave_sort64_u32(f2ord(mine == mine ? mine : __builtin_inff()));
                    const int j = (k + t - 1) / t;
                    const float B = ord2f((uint32_t)__shfl((int)sorted, j - 1, 64));
                    if (B < __builtin_inff()) {
                        const double qnorm_r =
                            (double)__int_as_float(__builtin_amdgcn_readlane(__float_as_int((float)my_qnorm), r));
                        const double E_r = err_E<METRIC>(qnorm_r, R, dd);
                        h = row_h<METRIC>(s_lim<METRIC>(bound_P<METRIC>((double)B, E_r, dd), E_r, dd), (double)qnf,
                                          qnorm_r, R);
                        const f2 w0 = d0 - a4.xy, w1 = d1 - a4.zw;
                        pm = ((w0.x >= h) | ((w0.y >= h) << 1) | ((w1.x >= h) << 2) | ((w1.y >= h) << 3)) & vmask;
                    }
                }
                const int lo_pos = (tile0 + tb + ti) * kTile + col;
                u64 key[4];
#pragma unroll
                for (int v = 0; v < 4; ++v) key[v] = ((u64)f2ord(sc[v]) << 32) | (uint32_t)(lo_pos + v);
                m_bufc[row] = s_append<RL>(lists + row * K2, bufs + row * 32, m_bufc[row], key[0], key[1], key[2],
                                           key[3], pm, a.stats);
            }
        }

        // ---- flush buffers, emit lists, publish bounds (wave-owned rows)
#pragma unroll 1
        for (int r = 0; r < RW; ++r) {
            const int row = wave * RW + r;
            const int bc = m_bufc[row];
            if (bc > 0) s_flush<RL>(lists + row * K2, bufs + row * 32, bc);
            const int pr = m_pair[row];
            if (pr >= 0) {
                u64 *dst = a.partial + ((int64_t)pr * a.nch_max + ch) * K2;
                for (int e = lane; e < K2; e += 64) dst[e] = lists[row * K2 + e];
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < RW && a.qbound && my_q >= 0) {
            const u64 kk = my_list[k - 1];
            if (kk != kEmptyKey) {
                const double P = bound_P<METRIC>((double)key_score(kk), my_E, dd);
                atomicMin(a.qbound + my_q, f2ord(__double2float_ru(P)));
            }
        }
        __syncthreads();
    }
}

// ---- merge: exact re-check of the survivors, final selection ---------------
struct SMergeArgs {
    const u64 *partial;
    const float *pE;  // NULL, or the screen's error bound per row list (tighter than the list-wide one)
    const int32_t *probe, *nch, *list_size, *tile_off, *ids;
    const int32_t *plive;  // NULL, or probe with the pairs k_pairs filtered out set to -1 (they have no lists)
    const float *Q, *Xr, *rmax;
    const uint32_t *qbound;
    float *D;
    int64_t *I;
    int64_t *ncand;
    int64_t nq, d, dpad;
    int n_lists, nprobe, k, K2, nch_max, bpc, dedup, per_partition;
    int groups, bpc_near;  // groups == 2: slot 0 pairs are virtual partition p, chunked by bpc_near
    int split;             // the lists came from the split-bf16 screen (its error model)
    int centred;           // ... on centred vectors: pqn[pair] = the row's norm, rmax the centred one
    const float *pqn;
    unsigned long long *stats;
    int unsorted;  // a list may hold its keys unsorted (k_screen_v): walk it to its first empty key
    const int32_t *head;  // head[19]: group 0's chunk size as the plan chose it
    // LIRA_OPT_RESCAN: 0 the merge re-scans a chunk whose list may have dropped a
    // candidate itself; 1 it only queues (q, slot, chunk, partition) in rq; 2 it takes
    // k_rescan's exact survivors rbuf[q][0 .. rcnt[q]) instead (rfall[q]: the queue
    // or the query's buffer overflowed -- its chunks are re-scanned here as in 0)
    int rmode, rq_cap, rcap;
    unsigned *rq_n, *rcnt, *rfall;
    int4 *rq;
    const u64 *rbuf;
    // k_screen_r's spill lists (NULL: none): keys its row lists evicted that may still
    // be needed, per query, (key lo, key hi, E bits, 0); scnt[q] > scap: overflowed
    const uint4 *spill;
    const unsigned *scnt;
    int scap;
};

// exact score of the candidate at storage row pos (search.cpp:253-269 order)
// (Xr: the row-major copy, so one lane reads its candidate contiguously).  q is
// wave-uniform (the merge's query row): read through the constant address space
// so its pieces come by scalar loads into SGPRs -- the 8 row pieces in flight then
// hold the VGPRs alone (k_smerge 128 -> 92 VGPRs, 4 -> 5 waves per SIMD; SIFT1M
// mixture merge 64 -> 49 us)
template <int METRIC, int U = 8>
__device__ __forceinline__ float exact_score(const float *q, const float *Xr, int64_t d, int pos) {
    const float *xp = Xr + (int64_t)pos * d;
    float acc = 0.0f;
    if ((d & 3) == 0 && ((uintptr_t)q & 15) == 0) {  // 16-B loads of the row, 8 in flight; the same sequential sum
        typedef float f4v __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(4))) f4v cf4;
        const float4 *x4 = (const float4 *)xp;
        cf4 *q4 = (cf4 *)q;
#pragma unroll U
        for (int64_t j = 0; j < d / 4; ++j) {
            const float4 xv = x4[j];
            const f4v qv = q4[j];
            if (METRIC == LIRA_METRIC_L2) {
                float df = qv.x - xv.x; acc = acc + df * df;
                df = qv.y - xv.y; acc = acc + df * df;
                df = qv.z - xv.z; acc = acc + df * df;
                df = qv.w - xv.w; acc = acc + df * df;
            } else {
                acc = acc + qv.x * xv.x;
                acc = acc + qv.y * xv.y;
                acc = acc + qv.z * xv.z;
                acc = acc + qv.w * xv.w;
            }
        }
        return METRIC == LIRA_METRIC_L2 ? acc : -acc;
    }
#pragma unroll 16
    for (int64_t j = 0; j < d; ++j) {
        if (METRIC == LIRA_METRIC_L2) {
            const float df = q[j] - xp[j];
            acc = acc + df * df;
        } else {
            acc = acc + q[j] * xp[j];
        }
    }
    return METRIC == LIRA_METRIC_L2 ? acc : -acc;
}

// ---- the MFMA screening kernel (default) ------------------------------------
// Same items, ring, thresholds and lists as k_screen (QR = 64 or 128 queries
// per item, QR/16 waves), but the dot
// products run on v_mfma_f32_16x16x4_f32, which on gfx950 is bitwise an
// fmaf chain in k order (cdna_hip_programming.md, FP32-input MFMA) -- the
// screen's error model holds unchanged -- and reaches the f32 peak that the
// VALU version (k_screen) cannot feed from LDS.  Wave w owns rows 16w..16w+15
// and all 256 candidates of a block as 16 tiles of 16 x 16: tile (t, i) has
// candidate 4j+i of block tile t in column j, so one ds_read_b128 per lane
// loads the B fragments of 4 tiles.  Lane l (g = l>>4, j = l&15) holds, per
// tile, rows 4g..4g+3 of column j: 16 candidates x 4 rows.
typedef float f4v __attribute__((ext_vector_type(4)));

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// SPLIT: the split-bf16 form.  X is then Xb (lira_abi.hip k_split_tiles): per
// tile and 16-dim chunk, [g 4][p 64][8 bf16] with g = 2 hl + h the hi/lo part
// of dims 8h..8h+7 of candidate 4 (p & 15) + (p >> 4), and QT the split layout
// of k_qstage<QR, true>.  One v_mfma_f32_16x16x32_bf16 per (tile, query part)
// and 16 dims: lane group g supplies k-slots 8g..8g+7 = (x part hl, dims h),
// the A operand the query's hi (then lo) part of the same dims, so the pair
// sums qh.(xh + xl) + ql.(xh + xl): 2 MFMAs of 16 cycles where the fp32 form
// needs 4 of 32, same LDS bytes, B fragments read once for both.  The error
// model is err_E(split = 1).
// SPLIT == 2 (LIRA_OPT_XHI): only the hi parts of x are staged and multiplied
// -- half the bytes and half the MFMAs -- one v_mfma_f32_16x16x32_bf16 per tile
// and 16 dims taking A = (qh, ql) of the 16 dims against B = (xh, xh); the
// bound widens by 2^-8 |q| R (err_E(split = 2)), so more candidates reach the
// exact re-check.
// SPLIT == 3 (LIRA_OPT_XHI = 2, hi x hi): only the hi parts of x AND of the
// queries, 32 dims per v_mfma_f32_16x16x32_bf16 (lane group g: chunk half g >>
// 1, dims 8 (g & 1) ..) and per ring slot: half the MFMAs, fragment reads and
// chunk barriers of SPLIT 2 and half its query bytes, at the bound
// err_E(split = 3) (+ ||q - qh|| (R + ||x - xh||), the row's qres from k_qstage).
template <int METRIC, int RL, int QR, int OCC, int SPLIT = 0>
__global__ __launch_bounds__(QR * 4, OCC) void k_screen_m(ScreenArgs a) {
    constexpr int NW = QR / 16, NT = QR * 4;  // waves of 16 rows each, threads
    typedef SSmem<QR, RL, true, SPLIT == 2, SPLIT == 3> S;
    constexpr int NSL = S::NSL;  // ring slots: 3 for hi-only x, else 2
    constexpr int K2 = S::K2, BC = S::BC;  // BC: survivor buffer keys per row
    constexpr int DK = SPLIT == 3 ? 2 * kSDK : kSDK;  // dims per staged chunk
    constexpr int ESPLIT = SPLIT;          // the error model's split mode
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *Xs = (float *)smem;  // [2] x {X: [4 tiles][16 dims][64], Q: [16 dims][64]}
    u64 *lists = (u64 *)(smem + S::kX);
    u64 *bufs = (u64 *)(smem + S::kX + S::kLists);
    int *meta = (int *)(smem + S::kX + S::kLists + S::kBufs);
    int *m_pair = meta + 16, *m_bufc = meta + 16 + QR;
    float2 *tri_s = (float2 *)(meta + 16 + 3 * QR);         // [2][QR]
    double *dq_s = (double *)(meta + 16 + 3 * QR + 4 * QR); // [QR][2]
    float2 *br_s = (float2 *)(dq_s + 2 * QR);               // [kBR] block radius ranges
    float *bres_s = (float *)(br_s + S::kBR);               // [kBR] (SPLIT 2) block hi residual bounds
    const bool TRI = METRIC == LIRA_METRIC_L2 && a.tstat != nullptr;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, cj = lane & 15;
    const int k = a.k;
    const double dd = (double)a.d;
    const float4 *Xg = (const float4 *)a.X;
    const uint32_t xs_lds = (uint32_t)(uintptr_t)(lds_void_t *)Xs;
    const int tstride = (int)a.dpad * (kTile / 4);
    const int nchunk = (int)(a.dpad / DK);

    long long t_0 = 0, t_1 = 0, t_2 = 0;  // (a.dbg & 8) phase clocks, thread 0
    long long t_ref = 0, t_chk = 0, t_sel = 0, t_x = 0, n_slow = 0, t_wt = 0;  // (a.dbg & 8) block-loop split
    // (phase clocks only in a -DLIRA_PHASE_CLOCKS build: their registers would
    // otherwise be live across the whole kernel)
    const bool clk = kPhaseClocks && (a.dbg & 8) && tid == 0;
    unsigned long long *const cnt = kPhaseClocks && (a.dbg & 8) ? nullptr : a.stats;  // (off while timing)
    __shared__ int xq[9];  // the XCD queues' bounds (k_plan)
    const int bpc_near_d = __builtin_amdgcn_readfirstlane(a.head[19]);  // group 0's chunk size (plan_body)
    int qx = 0, qtries = 0, nxt = -1;  // thread 0: its queue, the claimed next item
    int4 e_nxt = make_int4(0, 0, 0, 0);  // thread 0: the next item's table entry (loaded one item ahead)
    if (tid == 0) {
        for (int r = 0; r < 9; ++r) xq[r] = a.head[10 + r];
        qx = xcd_id();
        nxt = claim_item(a.head, xq, qx, qtries);
        if (nxt >= 0) e_nxt = a.itab[nxt];
    }  // thread 0: the claimed next item
    for (;;) {
        if (clk) t_0 = clock64();
        if (tid == 0) {
            // the next item is claimed, and its table entry loaded, one item
            // ahead (both complete under this item's work)
            const int item = nxt;
            const int ok = item >= 0;
            int4 e = make_int4(0, 0, 0, 0);
            if (ok) {
                e = e_nxt;
                nxt = claim_item(a.head, xq, qx, qtries);
                if (nxt >= 0) e_nxt = a.itab[nxt];
            }
            meta[0] = ok;
            meta[1] = e.x;
            meta[2] = e.y;
            meta[3] = e.z;
            meta[4] = e.w;
        }
        __syncthreads();
        if (!meta[0]) break;
        const int vp = __builtin_amdgcn_readfirstlane(meta[1]);  // virtual partition
        const int p = vp >= a.n_lists ? vp - a.n_lists : vp;
        const int ch = __builtin_amdgcn_readfirstlane(meta[3]);
        const int gqb = __builtin_amdgcn_readfirstlane(meta[4]);
        const bool QP = SPLIT == 3 && a.qpair;  // per-pair records (uniform)
        if (tid < QR) {
            if (QP) {
                const int qb = __builtin_amdgcn_readfirstlane(meta[2]);
                const int nval = a.cnt[vp] - qb * QR;
                m_pair[tid] = tid < nval ? a.qlist[a.qoff[vp] + qb * QR + tid] : -1;
            } else {
                m_pair[tid] = __float_as_int(a.QN[(int64_t)gqb * QR + tid].z);
            }
            m_bufc[tid] = 0;
        }
        for (int i = tid; i < QR * K2; i += NT) lists[i] = kEmptyKey;
        __syncthreads();

        const int tile0 = __builtin_amdgcn_readfirstlane(a.tile_off[p]);
        const int ntl = __builtin_amdgcn_readfirstlane(a.tile_off[p + 1]) - tile0;
        const int bpc = vp < a.n_lists && a.n_virt > a.n_lists ? bpc_near_d : a.bpc;
        const int tb_begin = ch * bpc * kSBT;
        const int tb_end = min(ntl, tb_begin + bpc * kSBT);
        const double R = (double)a.rmax[p];

        // lanes 0..15 of wave w hold row 16w + lane's threshold state
        const int my_row = wave * 16 + cj;
        const int qp_row = QP ? m_pair[my_row] : -1;
        const float4 qrec = QP ? (qp_row >= 0 ? a.QN[qp_row] : make_float4(0.0f, 0.0f, __int_as_float(-1), 0.0f))
                               : a.QN[(int64_t)gqb * QR + my_row];
        const int my_pair = __float_as_int(qrec.z);
        const int my_q = my_pair >= 0 ? my_pair / a.nprobe : -1;
        const double my_qn = (double)qrec.x, my_qnorm = (double)qrec.y;
        const double my_qres = SPLIT == 3 ? (double)(QP ? (qp_row >= 0 ? a.QE[qp_row] : 0.0f)
                                                        : a.QE[(int64_t)gqb * QR + my_row])
                                          : 0.0;
        // (QP) this lane's row (lane = row of the staged Q piece): its pair's hi parts in QH
        const int qh_row = QP ? max(m_pair[lane], 0) * (int)a.dpad : 0;
        const double my_E = err_E<METRIC>(my_qnorm, R, dd, ESPLIT, (double)a.dpad, a.centred, -1.0, my_qres);
        u64 *my_list = lists + my_row * K2;
        // this lane's 4 output rows 4g + reg: qn for the screened scores
        float qn_r[4];
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) qn_r[reg] = __shfl((float)my_qn, 4 * g + reg, 64);

        const float4 *qtg = (const float4 *)(a.QT + (int64_t)gqb * a.dpad * QR);
        // returns the DMA instructions this wave issued (the ring's vmcnt waits count them)
        auto stage = [&](int tb, int jc, int slot, int xpar) -> int {
            if (a.dbg & 4) return 0;  // timing experiment: no loads
            const int ntv = min(kSBT, tb_end - tb);
            const uint32_t base = xs_lds + (uint32_t)(slot * S::kStage);
            // X: 16 pieces of 1 KiB per chunk (tile pc >> 2, dims jc + 4(pc & 3)
            // .. +3; split: quarter (pc & 3) = part g); wave w moves pieces w, w + NW, ...
            // (SPLIT 2: the 8 hi pieces, quarters 0 and 1, tile stride 2 KiB)
            // (SPLIT 3: the 16 hi pieces of two 16-dim chunks, piece (t, chunk half
            // qq >> 1, quarter qq & 1), tile stride 4 KiB)
            constexpr int NP = SPLIT == 2 ? 8 : 16, QSH = SPLIT == 2 ? 1 : 2;
#pragma unroll
            for (int m = 0; m < NP / NW; ++m) {
                const int pc = wave + NW * m, t = pc >> QSH, qq = pc & ((1 << QSH) - 1);
                const int src = SPLIT == 3 ? (qq >> 1) * (kSDK * kTile / 4) + (qq & 1) * 64 : qq * 64;
                LIRA_SGLDS(Xg + (int64_t)(tile0 + tb + min(t, ntv - 1)) * tstride + jc * (kTile / 4) + src + lane,
                        __builtin_amdgcn_readfirstlane(base + (uint32_t)(t * S::kXT + qq * 1024)));
            }
            // Q: QR/16 pieces of 1 KiB, one per wave (SPLIT 3: the hi parts,
            // chunk half wave >> 1, quarter wave & 1; QR = 64)
            // (QP: gathered per row from QH -- dims jc + 16 (wave >> 1) + 8 (wave & 1) .. + 7
            // of row lane -- into the same LDS image)
            const int qsrc = SPLIT == 3 ? (wave >> 1) * (kSDK * QR / 4) + (wave & 1) * 64 : wave * 64;
            if (QP)
                LIRA_SGLDS(a.QH + qh_row + jc + 16 * (wave >> 1) + 8 * (wave & 1),
                           __builtin_amdgcn_readfirstlane(base + (uint32_t)S::kXS + (uint32_t)wave * 1024u));
            else
                LIRA_SGLDS(qtg + (int64_t)jc * (QR / 4) + qsrc + lane,
                           __builtin_amdgcn_readfirstlane(base + (uint32_t)S::kXS + (uint32_t)wave * 1024u));
            if (jc == 0 && wave == 0) {  // the block's xadj rides along (tiles past its end: masked on read)
                LIRA_SGLDS(a.xadj + (int64_t)(tile0 + tb + min(lane >> 4, ntv - 1)) * kTile + (lane & 15) * 4,
                           __builtin_amdgcn_readfirstlane(xs_lds + (uint32_t)(NSL * S::kStage + xpar * 1024)));
                return NP / NW + 2;
            }
            return NP / NW + 1;
        };

        // Triangle-inequality block skip (L2), as k_scan: ||q - x|| >= |
        // ||q - c_p|| - ||x - c_p|| | with per-tile bounds lo <= ||x - c_p||
        // <= hi, so a block whose radius range lies farther than rad_r from
        // ||q_r - c_p|| cannot hold a pair with exact score <= T_r, rad_r =
        // sqrt((T_r + d 2^-140) / (1 - (d+4) 2^-24)).  ||q_r - c_p|| in double:
        // row = 16w + (lane & 15), 4 lanes per row.
        // ||q_r - c_p|| from k_qstage (QN.w, within 1 ulp), widened by 2^-22
        if (TRI && g == 0) {
            const double dq = (double)qrec.w;
            dq_s[my_row * 2] = dq * (1.0 - 0x1p-22);
            dq_s[my_row * 2 + 1] = dq * (1.0 + 0x1p-22);
        }
        if (TRI) __builtin_amdgcn_wave_barrier();
        // Thresholds at a block's start (lanes 0..15: row 16w + lane): the
        // dot-product test h, and (TRI) the row's skip interval into tri_s[par]
        // (two parities: a wave refreshing the next block's never races one
        // still testing with this block's).
        // the query's published bound, read once per item (no global load on
        // the per-block path: the chunk loop's vmcnt(0) would wait for it)
        uint32_t pub = a.qbound && my_q >= 0
            ? __hip_atomic_load(a.qbound + my_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
        // with a.share: a row publishes its list's bound whenever it improves
        // and re-reads the query's bound for the next block (the load
        // completes under the next chunk's DMA wait), so concurrent items
        // of one query -- the chunks of its nearest partition above all --
        // prune with each other's progress
        uint32_t own_pub = ~0u;
        // Rb: the block's bound on ||x'|| (centred split screen with tile radius
        // ranges: max ||x - c|| over its tiles, widened for fl(x - c)), else the
        // list's R; the block's test threshold uses its own error bound Eb <= E
        // (a row's list bound P keeps the list-wide E: its keys come from every block)
        // E_run: the largest Eb of the blocks whose keys the list holds (every
        // key's screened score is within its block's Eb of the truth)
        double Rb = R, Eb = my_E, E_run = 0.0;
        bool c_ok = false;  // refresh's cache of the T-only terms
        double T_c = 0.0, A_c = 0.0;
        float2 ab_c = make_float2(-__builtin_inff(), __builtin_inff());
        auto refresh = [&](int par) {
            const u64 kk = my_list[k - 1];
            double T = kk == kEmptyKey ? __builtin_inf() : bound_P<METRIC>((double)key_score(kk), E_run, dd);
            if (a.share && a.qbound && my_q >= 0) {
                if (kk != kEmptyKey && lane < 16) {
                    const uint32_t b = f2ord(__double2float_ru(T));
                    if (b < own_pub) {
                        atomicMin(a.qbound + my_q, b);
                        own_pub = b;
                    }
                }
                if (pub != ~0u) T = fmin(T, (double)ord2f(pub));
                pub = __hip_atomic_load(a.qbound + my_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (pub != ~0u) {
                T = fmin(T, (double)ord2f(pub));
            }
            // the T-only parts (s_lim's division, the skip radius's sqrt) are
            // recomputed only when the row's bound moved (most blocks it does not)
            if (!c_ok || T != T_c) {
                c_ok = true;
                T_c = T;
                if (METRIC == LIRA_METRIC_L2) A_c = ((T + dd * 0x1p-140) / (1.0 - (dd + 4.0) * kU)) * (1.0 + 0x1p-50);
                if (TRI) {
                    ab_c = make_float2(-__builtin_inff(), __builtin_inff());  // never skip
                    const double F = 1.0 - (dd + 4.0) * kU;
                    if (my_pair < 0) {
                        ab_c = make_float2(__builtin_inff(), -__builtin_inff());  // no query: always
                    } else if (T < 1e300 && F > 0.5) {
                        const double rad = __builtin_sqrt((fmax(T, 0.0) + dd * 0x1p-140) / F) * (1.0 + 0x1p-40);
                        double A = dq_s[my_row * 2] - rad, B = dq_s[my_row * 2 + 1] + rad;
                        A -= __builtin_fabs(A) * 0x1p-50;
                        B += __builtin_fabs(B) * 0x1p-50;
                        ab_c = make_float2(__double2float_rd(A), __double2float_ru(B));
                    }
                }
            }
            // (s_lim<L2>(T, Eb) = A_c + Eb, the same double operations)
            const double lim = METRIC == LIRA_METRIC_L2 ? A_c + Eb : s_lim<METRIC>(T, Eb, dd);
            const float h = my_pair < 0 ? __builtin_inff() : row_h<METRIC>(lim, my_qn, my_qnorm, Rb);
            if (TRI && lane < 16) tri_s[par * QR + my_row] = ab_c;
            __builtin_amdgcn_wave_barrier();
            return h;
        };
        // radius range of the block at tile tb: staged in LDS for the item's
        // first kBR blocks (one round of loads per item), else from tstat
        const int nblk = (tb_end - tb_begin + kSBT - 1) / kSBT;
        const bool br_lds = TRI && nblk <= S::kBR;
        auto block_range_g = [&](int tb, float &lo, float &hi) {
            const int ntv = min(kSBT, tb_end - tb);
            lo = __builtin_inff();
            hi = -__builtin_inff();
#pragma unroll
            for (int i = 0; i < kSBT; ++i) {  // (independent loads in flight together)
                if (i < ntv) {
                    const float2 st = a.tstat[tile0 + tb + i];
                    lo = fminf(lo, st.x);
                    hi = fmaxf(hi, st.y);
                }
            }
        };
        // (SPLIT 2) the blocks' max ||x - hi(x)||: a tighter hi-only error bound than 2^-8 Rb
        const bool hres_on = (SPLIT == 2 || SPLIT == 3) && br_lds && a.tres != nullptr;
        if (br_lds) {
            for (int i = tid; i < nblk; i += NT) {
                float lo, hi;
                block_range_g(tb_begin + i * kSBT, lo, hi);
                br_s[i] = make_float2(lo, hi);
                if (hres_on) {
                    const int t0 = tb_begin + i * kSBT, nt = min(kSBT, tb_end - t0);
                    float m = 0.0f;
                    for (int u = 0; u < nt; ++u) m = fmaxf(m, a.tres[tile0 + t0 + u]);
                    bres_s[i] = m;
                }
            }
            __syncthreads();
        }
        auto block_range = [&](int tb, float &lo, float &hi) {
            if (br_lds) {
                const float2 v = br_s[(tb - tb_begin) / kSBT];
                lo = v.x;
                hi = v.y;
            } else {
                block_range_g(tb, lo, hi);
            }
        };
        // first block at or after t that some row may need (workgroup-uniform:
        // every wave tests all QR rows, QR/64 per lane, against the same LDS values)
        auto skip_from = [&](int t, int par) {
            if (TRI) {
                const float2 ab = lane < QR ? tri_s[par * QR + lane] : make_float2(__builtin_inff(), -__builtin_inff());
                const float2 ab2 = QR > 64 ? tri_s[par * QR + (QR > 64 ? 64 : 0) + lane]
                                           : make_float2(__builtin_inff(), -__builtin_inff());
                while (t < tb_end) {
                    float lo, hi;
                    block_range(t, lo, hi);
                    if (!__all((hi < ab.x || lo > ab.y) && (hi < ab2.x || lo > ab2.y))) break;
                    if (cnt && tid == 0) atomicAdd(cnt + 4, 1ull);
                    t += kSBT;
                }
            }
            return t;
        };

        // buffer fill of row 4 g + reg (this lane's group g), group-uniform
        int bcr[4] = {0, 0, 0, 0};
        int slot = 0;
        int tb = tb_begin;
        if (TRI) {
            refresh(1);
            __syncthreads();
            tb = skip_from(tb_begin, 1);
        }
        // The ring (NSL slots): the issuer stages chunk (itb, ijc) NSL - 1 chunks
        // ahead of the consumer, crossing into the next unskipped block with the
        // current block's skip intervals (looser than later ones: safe); the
        // blocks it enters queue up for the consumer (at most 2: nchunk >= 2).
        int itb = tb, ijc = 0, islot = 0, par_i = 1, iblk = 0;  // iblk: the issuer's block count
        int q_n = 0, q_0 = tb_end, q_1 = tb_end;  // queued block starts
        int n_cur = 0, n_nxt = 0;                 // this wave's DMAs of the chunks after the consumer's
        auto issue = [&]() -> int {
            if (itb >= tb_end) return 0;
            const int n = stage(itb, ijc * DK, islot, iblk & 1);
            islot = islot + 1 == NSL ? 0 : islot + 1;
            if (++ijc == nchunk) {
                ijc = 0;
                ++iblk;
                itb = skip_from(itb + kSBT, par_i);
                if (q_n == 0) q_0 = itb; else q_1 = itb;
                ++q_n;
            }
            return n;
        };
        n_cur = issue();
        if (NSL == 3) n_nxt = issue();

        if (clk) t_1 = clock64();
        auto pop = [&]() {  // the next block the issuer entered
            const int v = q_0;
            q_0 = q_1;
            --q_n;
            return v;
        };
#pragma unroll 1
        for (int bi = 0; tb < tb_end; ++bi, tb = pop()) {
            if (clk) t_x = clock64();
            const int ntv = min(kSBT, tb_end - tb);
            float blo = 0.0f, bhi = 0.0f;
            if (TRI) block_range(tb, blo, bhi);
            if (TRI && SPLIT && a.centred) {
                Rb = fmin(R, (double)bhi * (1.0 + 0x1p-20));
                const double hr = hres_on ? (double)bres_s[(tb - tb_begin) / kSBT] : -1.0;
                Eb = Rb < R || hres_on ? err_E<METRIC>(my_qnorm, Rb, dd, ESPLIT, (double)a.dpad, a.centred, hr, my_qres)
                                       : my_E;
            }
            const float h_l = refresh(bi & 1);
            E_run = fmax(E_run, Eb);  // (this block's keys join the list below)
            // a wave whose 16 rows all skip the block (or hold no query)
            // computes nothing for it
            bool wdead = !__any(lane < 16 && my_pair >= 0);
            if (TRI && !wdead) {
                const float2 ab = tri_s[(bi & 1) * QR + wave * 16 + cj];
                wdead = __all(bhi < ab.x || blo > ab.y);
            }

            f4v acc[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = (f4v)(0.0f);
            if (clk) {
                const long long t = clock64();
                t_ref += t - t_x;
                t_x = t;
            }

            par_i = bi & 1;  // the issuer's skip test uses this block's intervals
#pragma unroll 1
            for (int c = 0; c < nchunk; ++c) {
                const long long t_w0 = clk ? clock64() : 0;
                // this chunk's DMAs landed (the ones issued after it may stay in
                // flight: vmcnt counts this wave's vector-memory ops in order)
                if (NSL == 3 && n_nxt > 0) {
                    if (n_nxt >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    else if (n_nxt == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                    else if (n_nxt == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __syncthreads();  // ... in every wave; and the slot issued next is free
                if (clk) t_wt += clock64() - t_w0;
                n_cur = n_nxt;
                n_nxt = issue();
                if (NSL == 2) {
                    n_cur = n_nxt;
                    n_nxt = 0;
                }
                if (SPLIT == 3 && !wdead && !(a.dbg & 1)) {
                    const char *sb = (const char *)Xs + slot * S::kStage;
                    // A: the rows' qh of dims 8g .. 8g + 7 of the slot's 32; B: xh of the same dims
                    const bf16x8 aq = *(const bf16x8 *)(sb + S::kXS + ((g * QR + wave * 16 + cj) << 4));
                    bf16x8 bv[16];
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            bv[t * 4 + i] = *(const bf16x8 *)(sb + t * S::kXT + ((g * 64 + i * 16 + cj) << 4));
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, bv[i], acc[i], 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 9, 0);  // DS reads
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMAs
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                } else if (SPLIT == 2 && !wdead && !(a.dbg & 1)) {
                    const char *sb = (const char *)Xs + slot * S::kStage;
                    // all 17 fragment reads first, then the 16 MFMAs (pinned by sched
                    // groups: left to itself hipcc serialises read -> wait -> MFMA)
                    const bf16x8 aq = *(const bf16x8 *)(sb + S::kXS + ((g * QR + wave * 16 + cj) << 4));
                    bf16x8 bv[16];
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            bv[t * 4 + i] = *(const bf16x8 *)(sb + t * S::kXT + (((g & 1) * 64 + i * 16 + cj) << 4));
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, bv[i], acc[i], 0, 0, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 9, 0);  // DS reads
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMAs
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                } else if (SPLIT && !wdead && !(a.dbg & 1)) {
                    const char *sb = (const char *)Xs + slot * S::kStage;
                    const bf16x8 a_hi = *(const bf16x8 *)(sb + S::kXS + (((g & 1) * QR + wave * 16 + cj) << 4));
                    const bf16x8 a_lo = *(const bf16x8 *)(sb + S::kXS + (((2 + (g & 1)) * QR + wave * 16 + cj) << 4));
                    bf16x8 bv[16];
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            bv[t * 4 + i] = *(const bf16x8 *)(sb + t * S::kXT + ((g * 64 + i * 16 + cj) << 4));
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            acc[t * 4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_hi, bv[t * 4 + i], acc[t * 4 + i], 0, 0, 0);
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            acc[t * 4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_lo, bv[t * 4 + i], acc[t * 4 + i], 0, 0, 0);
                    }
                    // the next tile's B fragments in flight under this tile's 8 MFMAs
                    __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);  // A hi / lo + tiles 0, 1
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
                } else if (!SPLIT && !wdead && !(a.dbg & 1)) {
                    const float *sb = (const float *)((const char *)Xs + slot * S::kStage);
                    const float *xb = sb + g * kTile + 4 * cj;                   // + t*1024 + 4s*64
                    const float *qa = sb + S::kXS / 4 + g * QR + wave * 16 + cj;  // + 4s*64
#pragma unroll
                    for (int s4 = 0; s4 < kSDK / 4; ++s4) {
                        const float av = qa[s4 * 4 * QR];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const f4 bv = *(const f4 *)(xb + t * (kSDK * kTile) + s4 * 4 * kTile);
                            acc[t * 4 + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv.x, acc[t * 4 + 0], 0, 0, 0);
                            acc[t * 4 + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv.y, acc[t * 4 + 1], 0, 0, 0);
                            acc[t * 4 + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv.z, acc[t * 4 + 2], 0, 0, 0);
                            acc[t * 4 + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv.w, acc[t * 4 + 3], 0, 0, 0);
                        }
                    }
                }
                slot = slot + 1 == NSL ? 0 : slot + 1;
            }
            if (cnt && lane == 0) {
                if (wave == 0) atomicAdd(cnt + 2, 1ull);
                if (!wdead) atomicAdd(cnt + 0, 16ull * kSBT * kTile);  // (row, candidate) pairs screened
            }
            if (clk) {
                const long long t = clock64();
                t_chk += t - t_x;
                t_x = t;
            }
            if (wdead || (a.dbg & 2)) continue;
            // xadj of my 16 candidates: tile t, i = 0..3 (+inf: padding / past the block)
            f4 xa[4];
            {
                const float *xs = (const float *)((const char *)Xs + NSL * S::kStage + (bi & 1) * 1024);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    xa[t] = t < ntv ? *(const f4 *)(xs + t * kTile + 4 * cj) : (f4)(__builtin_inff());
            }

            float h_r[4];
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) h_r[reg] = from_row_lane(h_l, reg, g);

            // ---- selection: per output register reg, lane group g holds row
            // 4g + reg's 16 candidates; the four rows of a reg go together
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                float h = h_r[reg];
                float wv[16];  // fl(dot - xadj) of my 16 candidates
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const f2 w0 = (f2){acc[t * 4 + 0][reg], acc[t * 4 + 1][reg]} - xa[t].xy;
                    const f2 w1 = (f2){acc[t * 4 + 2][reg], acc[t * 4 + 3][reg]} - xa[t].zw;
                    wv[4 * t + 0] = w0.x;
                    wv[4 * t + 1] = w0.y;
                    wv[4 * t + 2] = w1.x;
                    wv[4 * t + 3] = w1.y;
                }
                // one compare per lane first (max3 tree; fmaxf drops NaN, which
                // never passes the per-candidate test either)
                const float m01 = fmaxf(fmaxf(wv[0], wv[1]), wv[2]), m02 = fmaxf(fmaxf(wv[3], wv[4]), wv[5]);
                const float m03 = fmaxf(fmaxf(wv[6], wv[7]), wv[8]), m04 = fmaxf(fmaxf(wv[9], wv[10]), wv[11]);
                const float m05 = fmaxf(fmaxf(wv[12], wv[13]), wv[14]);
                const float mx = fmaxf(fmaxf(fmaxf(m01, m02), m03), fmaxf(fmaxf(m04, m05), wv[15]));
                if (!__any(mx >= h)) continue;  // wave-uniform: none of the four rows has a candidate
                if (clk) ++n_slow;
                // passing candidates; padding (xadj = +inf: wv = -inf) never, as
                // h is clamped to the lowest finite value (one compare per candidate)
                const float hp = fmaxf(h, -3.40282347e38f);
                int pm = 0;
#pragma unroll
                for (int i = 0; i < 16; ++i) pm |= (wv[i] >= hp) << i;
                // screened score of candidate i (L2: qn + 2 xadj - 2 dot; IP: -dot)
                auto score = [&](int i) {
                    const float av = xa[i >> 2][i & 3], dv = acc[i][reg];
                    return METRIC == LIRA_METRIC_L2 ? __builtin_fmaf(-2.0f, dv, qn_r[reg] + 2.0f * av) : -dv;
                };
                if (__any(h == -__builtin_inff()) && k <= 64) {
                    // a row without a bound yet: t = ceil(k/16) smallest of each
                    // of its 16 lanes, j = ceil(k/t) <= 16 over those lanes
                    float m4[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const float sv = score(i);
                        float v = xa[i >> 2][i & 3] != __builtin_inff() && sv == sv ? sv : __builtin_inff();
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const float lo = fminf(m4[u], v), hi = fmaxf(m4[u], v);
                            m4[u] = lo;
                            v = hi;
                        }
                    }
                    const int t = (k + 15) / 16;
                    uint32_t key16 = f2ord(t <= 1 ? m4[0] : t == 2 ? m4[1] : t == 3 ? m4[2] : m4[3]);
#pragma unroll
                    for (int size = 2; size <= 16; size <<= 1)  // ascending sort within each 16-lane group
#pragma unroll
                        for (int stride = size >> 1; stride > 0; stride >>= 1) {
                            const uint32_t o = xor_u32(key16, stride);
                            const bool lower = (cj & stride) == 0, asc = (cj & size) == 0;
                            key16 = (lower == asc) ? min(key16, o) : max(key16, o);
                        }
                    const int j = (k + t - 1) / t;
                    const float B = ord2f((uint32_t)__shfl((int)key16, 16 * g + j - 1, 64));
                    if (h == -__builtin_inff() && B < __builtin_inff()) {
                        const double qnorm_r = (double)__shfl((float)my_qnorm, 4 * g + reg, 64);
                        const double qres_r = SPLIT == 3 ? (double)__shfl((float)my_qres, 4 * g + reg, 64) : 0.0;
                        // (bound from this block's keys: its own error bound serves both)
                        const double E_r = err_E<METRIC>(qnorm_r, Rb, dd, ESPLIT, (double)a.dpad, a.centred,
                                                         hres_on ? (double)bres_s[(tb - tb_begin) / kSBT] : -1.0, qres_r);
                        h = row_h<METRIC>(s_lim<METRIC>(bound_P<METRIC>((double)B, E_r, dd), E_r, dd),
                                          (double)qn_r[reg], qnorm_r, Rb);
                        int pm2 = 0;
#pragma unroll
                        for (int i = 0; i < 16; ++i) pm2 |= (acc[i][reg] - xa[i >> 2][i & 3] >= h) << i;
                        pm &= pm2;
                    }
                }
                // append: lane group g adds its passing keys to row 4g + reg's
                // buffer, lanes in order (offsets from a 16-lane prefix sum of
                // the lanes' counts), each lane its own keys in column order --
                // no per-column ballots.  A row whose buffer cannot take them is
                // merged into its list first; more than BC keys (first blocks,
                // loose bounds) go in rounds of BC, merging between rounds.  One
                // merge site, so the reg loop still unrolls (acc[v][reg] static).
                {
                    const int row = wave * 16 + 4 * g + reg;
                    const int bc0 = bcr[reg];  // (group-uniform)
                    const int n_l = __builtin_popcount(pm);
                    const int inc = row16_incl_scan(n_l);  // inclusive prefix over the group's 16 lanes
                    const int rowtot = row16_total(inc);
                    const bool pre = bc0 > 0 && bc0 + rowtot > BC;  // merge the buffer first
                    const int total = (pre ? 0 : bc0) + rowtot;    // the row's keys in buffer order
                    const int base = (pre ? 0 : bc0) + inc - n_l;  // rank of my first key
                    for (int r0 = 0;; r0 += BC) {
                        // round 0: rows merging before appending; round r: rows
                        // whose previous window filled
                        u64 fl = __ballot((r0 == 0 ? pre : total > r0) && cj == 0);
                        while (fl) {
                            const int gg = __builtin_ctzll(fl) >> 4;
                            fl &= fl - 1;
                            const int r = wave * 16 + 4 * gg + reg;
                            s_flush<RL>(lists + r * K2, bufs + r * BC, r0 == 0 ? __builtin_amdgcn_readlane(bc0, 16 * gg) : BC);
                        }
                        // each lane walks its own passing candidates (usually 0 or 1):
                        // a 16-way select picks the accumulator, so only those are
                        // scored (scoring all 16 unconditionally was ~150 VALU per pass)
                        int rank = base, pmv = pm;
                        while (pmv) {
                            const int v = __builtin_ctz(pmv);
                            pmv &= pmv - 1;
                            if (rank >= r0 && rank < r0 + BC) {
                                float dv = acc[0][reg], av = xa[0][0];
#pragma unroll
                                for (int i = 1; i < 16; ++i)
                                    if (v == i) {
                                        dv = acc[i][reg];
                                        av = xa[i >> 2][i & 3];
                                    }
                                const float sc = METRIC == LIRA_METRIC_L2
                                                     ? __builtin_fmaf(-2.0f, dv, qn_r[reg] + 2.0f * av) : -dv;
                                bufs[row * BC + rank - r0] =
                                    ((u64)f2ord(sc) << 32) | (uint32_t)((tile0 + tb + (v >> 2)) * kTile + 4 * cj + (v & 3));
                            }
                            ++rank;
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (!__any(total - r0 > BC)) break;
                    }
                    bcr[reg] = total <= BC ? total : total - BC * ((total - 1) / BC);
                    if (cj == 0 && cnt && rowtot) atomicAdd(cnt + 7, (unsigned long long)rowtot);
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (clk) t_sel += clock64() - t_x;
        }

        if (clk) t_2 = clock64();
        if (cj == 0) {  // the rows' buffer fills, from registers to LDS
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) m_bufc[wave * 16 + 4 * g + reg] = bcr[reg];
        }
        __builtin_amdgcn_wave_barrier();
        // ---- flush buffers, emit lists, publish bounds (wave-owned rows);
        // buffers flushed two rows per network pass (one row per half-wave:
        // the per-item epilogue was ~8 % of the screen's cycles on SIFT1M latent)
        // A row whose list is still empty and whose buffer holds fewer than k keys
        // is NOT merged: its keys go out unsorted, marked by kUnsortedMark in the
        // list's last slot (k_smerge then walks the list to its first empty key).
        // Merging could not give it a k-th key to publish either, so the bounds
        // are unchanged; the merges were most of the item epilogue (SIFT1M
        // mixture at 1.25 k queries: 16 % of the screen's cycles).
        {
            const int nb = lane < 16 ? m_bufc[wave * 16 + lane] : 0;
            u64 pend = __ballot(lane < 16 && nb > 0 && (nb >= k || lists[(wave * 16 + lane) * K2] != kEmptyKey));
            while (pend) {
                const int ra = __builtin_ctzll(pend);
                pend &= pend - 1;
                int rb = -1;
                if (pend) {
                    rb = __builtin_ctzll(pend);
                    pend &= pend - 1;
                }
                const int rowa = wave * 16 + ra, na = __builtin_amdgcn_readlane(nb, ra);
                if (rb >= 0) {
                    const int rowb = wave * 16 + rb, nbb = __builtin_amdgcn_readlane(nb, rb);
                    s_flush2<RL>(lists + rowa * K2, bufs + rowa * BC, na, lists + rowb * K2, bufs + rowb * BC, nbb);
                } else {
                    s_flush<RL>(lists + rowa * K2, bufs + rowa * BC, na);
                }
            }
        }
#pragma unroll 1
        for (int r = 0; r < 16; ++r) {
            const int row = wave * 16 + r;
            const int pr = m_pair[row];
            if (pr >= 0) {
                u64 *dst = a.partial + ((int64_t)pr * a.nch_max + ch) * K2;
                const int nb = m_bufc[row];
                const bool uns = nb > 0 && nb < k && lists[row * K2] == kEmptyKey;  // (not merged above)
                for (int e = lane; e < K2; e += 64)
                    dst[e] = !uns ? lists[row * K2 + e] : e < nb ? bufs[row * BC + e] : e == K2 - 1 ? kUnsortedMark : kEmptyKey;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < 16 && my_pair >= 0 && a.pE)  // (>= every listed key's own block bound)
            a.pE[(int64_t)my_pair * a.nch_max + ch] = __double2float_ru(fmax(E_run, 0x1p-126));
        if (lane < 16 && a.qbound && my_q >= 0) {
            const u64 kk = my_list[k - 1];
            if (kk != kEmptyKey) {
                const double P = bound_P<METRIC>((double)key_score(kk), E_run, dd);
                atomicMin(a.qbound + my_q, f2ord(__double2float_ru(P)));
            }
        }
        __syncthreads();
        if (clk && a.stats) {  // timing experiment: cycles per phase
            const long long t_3 = clock64();
            atomicAdd(a.stats + 1, (unsigned long long)(t_1 - t_0));
            atomicAdd(a.stats + 3, (unsigned long long)(t_2 - t_1));
            atomicAdd(a.stats + 6, (unsigned long long)(t_3 - t_2));
            // the block loop's split (wave 0): refresh + skip test, chunk loop
            // (staging + MFMA), selection (blocks that reach it), slow-path regs
            atomicAdd(a.stats + 0, (unsigned long long)t_ref);
            atomicAdd(a.stats + 2, (unsigned long long)t_chk);
            atomicAdd(a.stats + 4, (unsigned long long)t_sel);
            atomicAdd(a.stats + 7, (unsigned long long)n_slow);
            atomicAdd(a.stats + 5, (unsigned long long)t_wt);  // of which: waits + barriers at chunk starts
            t_ref = t_chk = t_sel = n_slow = t_wt = 0;
        }
    }
}

// ---- seed: a finite starting bound for every query ----------------------
// One wave per query: exact scores of the first kSeedTiles tiles (256 rows) of its first
// probed partition; with t = ceil(k/64) smallest per lane and j = ceil(k/t),
// the j-th smallest lane value has >= k real (distinct) candidates at or below
// it, so it bounds the query's final k-th exact score.  Written to qbound
// before k_screen, so no item starts unbounded (which would push a whole
// first block per row through the selection).
static constexpr int kSeedTiles = 4;
// The same bound from the fp32 tiles where the index keeps them (one wave per
// query, lane = candidate: each dim of a tile is one coalesced 256-B row).
// NT tiles: 2 for k <= 32 (measured SIFT1M mixture: plan 0.217 -> 0.164 ms,
// scan +0.02 ms), else NT.
// the seed bound of query q (wave-uniform; +inf: none): k exact candidates of
// its slot-0 list, the first NT tiles, score <= the returned value
template <int METRIC, int NT>
__device__ __forceinline__ float seed_bound(const float *Q, const int32_t *probe, int nprobe, int n_lists,
                                           const int32_t *tile_off, const int32_t *ids, const float *X, int64_t d,
                                           int64_t dpad, int64_t q, int k) {
    const int lane = threadIdx.x & 63;
    const int p = probe[q * nprobe];
    if (p < 0 || p >= n_lists) return __builtin_inff();
    const int tile0 = tile_off[p], nt = min(NT, tile_off[p + 1] - tile0);
    if (nt <= 0) return __builtin_inff();
    const float *qrow = Q + q * d;
    const float *xt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) xt[t] = X + (int64_t)(tile0 + min(t, nt - 1)) * dpad * kTile + lane;
    float acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0.0f;
    for (int64_t j0 = 0; j0 < d; j0 += 64) {
        const float qv = j0 + lane < d ? qrow[j0 + lane] : 0.0f;
        const int nj = (int)min<int64_t>(64, d - j0);
        if (nj == 64) {
            // two tiles per packed fp32 op (v_pk_add_f32 / v_pk_mul_f32 round
            // each half like the scalar ops: the same per-lane sums)
            f2 acc2[NT / 2 > 0 ? NT / 2 : 1];
#pragma unroll
            for (int t = 0; t < NT / 2; ++t) acc2[t] = (f2){acc[2 * t], acc[2 * t + 1]};
#pragma unroll 16
            for (int jj = 0; jj < 64; ++jj) {
                const f2 qj = (f2)(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv), jj)));
#pragma unroll
                for (int t = 0; t < NT / 2; ++t) {
                    const f2 xv = {xt[2 * t][(j0 + jj) * kTile], xt[2 * t + 1][(j0 + jj) * kTile]};
                    if (METRIC == LIRA_METRIC_L2) {
                        const f2 df = qj - xv;
                        acc2[t] = acc2[t] + df * df;
                    } else {
                        acc2[t] = acc2[t] + qj * xv;
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < NT / 2; ++t) {
                acc[2 * t] = acc2[t].x;
                acc[2 * t + 1] = acc2[t].y;
            }
            if (NT & 1) {  // (an odd tile: scalar; 64 loads in flight -- GIST1M's one seed tile
                           // of 960 dims ran as 60 dependent rounds of 16 at unroll 16: 39 -> 31 us)
#pragma unroll 64
                for (int jj = 0; jj < 64; ++jj) {
                    const float qj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv), jj));
                    const float xv = xt[NT - 1][(j0 + jj) * kTile];
                    if (METRIC == LIRA_METRIC_L2) {
                        const float df = qj - xv;
                        acc[NT - 1] = acc[NT - 1] + df * df;
                    } else {
                        acc[NT - 1] = acc[NT - 1] + qj * xv;
                    }
                }
            }
        } else {
            for (int jj = 0; jj < nj; ++jj) {
                const float qj = __shfl(qv, jj, 64);
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const float xv = xt[t][(j0 + jj) * kTile];
                    if (METRIC == LIRA_METRIC_L2) {
                        const float df = qj - xv;
                        acc[t] = acc[t] + df * df;
                    } else {
                        acc[t] = acc[t] + qj * xv;
                    }
                }
            }
        }
    }
    float m[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};  // 4 smallest
#pragma unroll
    for (int u = 0; u < NT; ++u) {
        float sc = METRIC == LIRA_METRIC_L2 ? acc[u] : -acc[u];
        if (u >= nt || ids[(tile0 + u) * kTile + lane] < 0 || !(sc == sc)) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float lo = fminf(m[i], sc), hi = fmaxf(m[i], sc);
            m[i] = lo;
            sc = hi;
        }
    }
    const int t = (k + 63) / 64;
    if (t > 4) return __builtin_inff();
    const float mine = t == 1 ? m[0] : t == 2 ? m[1] : t == 3 ? m[2] : m[3];
    const uint32_t sorted = wave_sort64_u32(f2ord(mine));
    const int j = (k + t - 1) / t;
    return ord2f((uint32_t)__shfl((int)sorted, j - 1, 64));
}

// PAIRS: the query's per-pair records and partition filter (pair_record, as
// k_pairs) right after its seed, with the seed bound from registers -- one
// launch and one read of the query row fewer; qbound is then written for
// every query (~0: no bound), so the caller needs no fill.
struct SeedPairs {
    const float *pivot;
    int centred;
    const float2 *lstat;
    int32_t *probe_live;
    float4 *QN;
    float *QE;
    float *pqn;
    uint16_t *QH;
    const int32_t *list_size;  // (non-null) estimate the blocks each pair will screen (pair_record,
    const float2 *lsamp;       //   from lira_index::lsamp) on every 8th query, summed into
    unsigned int *work;        //   work[(q / 8) % 64] (the plan adds the 64 up and scales by 8)
    // (k_seed_p, non-null cnt) k_count's counts: every live pair adds 1 to its virtual
    // partition's counter (groups == 2: slot 0 -> p, else n_lists + p) in its XCD's
    // replica cnt[xcd * nv + v] (device-scope atomics on one address serialise: one
    // counter per partition cost the 10 k-query seed 19 us), no rank taken; k_plan_fill
    // sums the replicas; a probe id >= n_lists sets err
    int32_t *cnt = nullptr;
    int nv = 0;
    int32_t *err = nullptr;
    int groups = 1;
};
template <int METRIC, int NT = kSeedTiles, bool PAIRS = false>
__global__ __launch_bounds__(256) void k_seed_t(const float *Q, const int32_t *probe, int nprobe, int n_lists,
                                                const int32_t *tile_off, const int32_t *ids, const float *X,
                                                int64_t d, int64_t dpad, int64_t nq, int k, uint32_t *qbound,
                                                SeedPairs sp) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const float B = seed_bound<METRIC, NT>(Q, probe, nprobe, n_lists, tile_off, ids, X, d, dpad, q, k);
    const uint32_t qb = B < __builtin_inff() ? f2ord(B) : ~0u;
    if (PAIRS) {
        if (lane == 0) qbound[q] = qb;
        // the work estimate on every 8th query (a statistic: the plan scales it by 8)
        const bool samp = sp.work && (q & 7) == 0;
        int est = 0;
        for (int s0 = 0; s0 < nprobe; s0 += 4) {
            const int slot = s0 + (lane >> 4);
            const bool valid = slot < nprobe;
            const int64_t pair = q * nprobe + (valid ? slot : 0);
            const int praw = valid ? probe[pair] : -1;
            est += pair_record(Q, d, pair, valid, praw, nprobe, n_lists, sp.pivot, sp.centred, sp.lstat, qb,
                               sp.probe_live, sp.QN, sp.QE, sp.pqn, sp.QH, dpad, samp ? sp.list_size : nullptr,
                               sp.lsamp);
        }
        if (samp) {  // lanes 0, 16, 32, 48 hold their pair groups' sums
            const int tot = __builtin_amdgcn_readlane(est, 0) + __builtin_amdgcn_readlane(est, 16) +
                            __builtin_amdgcn_readlane(est, 32) + __builtin_amdgcn_readlane(est, 48);
            if (lane == 0 && tot) atomicAdd(sp.work + ((q >> 3) & 63), (unsigned)tot);
        }
    } else if (lane == 0 && qb != ~0u) {
        qbound[q] = qb;
    }
}

// One (query, slot) pair's record sums over G lanes, lane sub owning the contiguous
// dims [sub D, sub D + D) (D = ceil(d / G) rounded up to 4): s = sum fl(q - c)^2 (L2
// centred) or q^2, e = the hi residuals', t = sum (q - c)^2 (L2) or q.c (IP, centred
// == 2), all in double; the QH row (hi(q') in bf16, zero past d) written 4 at a time.
// Every lane returns the pair's totals (pair_record's values up to the double sums'
// order).  p < 0: zeros, nothing written.
template <int G>
__device__ __forceinline__ void pair_sums_run(const float *qrow, const float *pv, int64_t d, int64_t dpad, int64_t pair,
                                              int sub, int p, uint16_t *QH, int centred, double &s, double &t,
                                              double &e) {
    const int64_t D = ((d + G - 1) / G + 3) & ~(int64_t)3;
    const int64_t j0 = sub * D, j1 = min<int64_t>(d, j0 + D);
    s = t = e = 0.0;
    if (p >= 0) {
        uint16_t *qh = QH ? QH + pair * dpad : nullptr;
        const bool cen = centred == 1, ipm = centred == 2;
        auto one = [&](float x, float cv, uint32_t &hb) {
            const float sv = cen ? x - cv : x;
            hb = bf16_rne_sat(sv);
            const double xc = (double)sv;
            s = __builtin_fma(xc, xc, s);
            const double rr = (double)(sv - __uint_as_float(hb << 16));
            e = __builtin_fma(rr, rr, e);
            if (ipm) {
                t = __builtin_fma((double)x, (double)cv, t);
            } else {
                const double df = (double)x - (double)cv;
                t = __builtin_fma(df, df, t);
            }
        };
        if ((d & 3) == 0) {  // 16-B loads (rows 16-B aligned), 4 bf16 per 8-B store
#pragma unroll 4
            for (int64_t j = j0; j < j1; j += 4) {
                const float4 x4 = *(const float4 *)(qrow + j), c4 = *(const float4 *)(pv + j);
                uint32_t h0, h1, h2, h3;
                one(x4.x, c4.x, h0);
                one(x4.y, c4.y, h1);
                one(x4.z, c4.z, h2);
                one(x4.w, c4.w, h3);
                if (qh) *(uint2 *)(qh + j) = make_uint2(h0 | (h1 << 16), h2 | (h3 << 16));
            }
        } else {
            for (int64_t j = j0; j < j1; ++j) {
                uint32_t h;
                one(qrow[j], pv[j], h);
                if (qh) qh[j] = (uint16_t)h;
            }
        }
        if (qh) {  // zeros from d to dpad: in this lane's run, then past all G runs
            for (int64_t j = max(d, j0); j < min(j0 + D, dpad); ++j) qh[j] = 0;
            for (int64_t j = G * D + sub; j < dpad; j += G) qh[j] = 0;
        }
    }
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) {  // within the pair's lanes
        s += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, s), m));
        t += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, t), m));
        e += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, e), m));
    }
}

// k_seed_t<L2, NT, true> with all of the query's pair records in ONE round
// (k_seed_p): G = 64 / nprobe_pow2 lanes per (query, slot) pair, each lane a
// contiguous run of D dims (16-B loads of q and the pivot, 8-B stores of 4 bf16
// of QH), so the nprobe pairs' loads are in flight together and the filter runs
// in every pair's lanes at once.  k_seed_t walked the pairs 4 at a time (16 lanes
// each, dims strided by 16): at nprobe 8 two rounds of probe -> pivot -> reduce
// -> filter chains after the seed's own, about 35 of its 55 us per 10 k SIFT1M
// queries (seed tiles 1 / 2 / 4: 46 / 56 / 101 us).  The records are the same
// values as pair_record's (double sums in another order: fl() of the same exact
// sum up to the double rounding, which the screen's error model absorbs -- the
// results never depend on it); the seed bound is seed_bound's, bit for bit.
// (110 VGPRs, 4 waves per SIMD; capped at 78 for 6 -- 2 of the 16-B record loads in flight
// instead of 4 -- it ran 51 -> 100 us per 10 k queries: the waves' load chains, not
// their number, set its time)
template <int NT, int G>
__global__ __launch_bounds__(256) void k_seed_p(const float *Q, const int32_t *probe, int nprobe, int n_lists,
                                                const int32_t *tile_off, const int32_t *ids, const float *X,
                                                int64_t d, int64_t dpad, int64_t nq, int k, uint32_t *qbound,
                                                SeedPairs sp) {
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "lanes per pair");
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;
    const int slot = lane / G, sub = lane % G;
    const bool valid = slot < nprobe;
    const int64_t pair = q * nprobe + (valid ? slot : 0);
    const int praw = valid ? probe[pair] : -1;
    const int p = praw < n_lists ? praw : -1;
    const float *qrow = Q + q * d;
    const bool est_on = sp.work && (q & 7) == 0 && p >= 0;
    // (estimate) the 16 sample tiles of the list, 16 / G per lane
    float2 ts[16 / G];
#pragma unroll
    for (int i = 0; i < 16 / G; ++i) ts[i] = est_on ? sp.lsamp[p * 16 + sub + G * i] : make_float2(0.0f, 0.0f);
    const int lsz = est_on ? sp.list_size[p] : 0;
    double s, t, e;
    pair_sums_run<G>(qrow, p >= 0 ? sp.pivot + (int64_t)p * d : nullptr, d, dpad, pair, sub, p, sp.QH, sp.centred, s, t,
                     e);
    // the seed bound (seed_bound: the first NT tiles of slot 0's list)
    const float B = seed_bound<LIRA_METRIC_L2, NT>(Q, probe, nprobe, n_lists, tile_off, ids, X, d, dpad, q, k);
    const uint32_t qb = B < __builtin_inff() ? f2ord(B) : ~0u;
    if (lane == 0) qbound[q] = qb;
    // the filter (pair_record's triangle test), in every lane of every pair
    int live = p;
    const float dq = (float)__builtin_sqrt(t);
    const double qnd = __builtin_sqrt(s);
    float fa = -__builtin_inff(), fb = __builtin_inff();
    if (p >= 0 && sp.lstat && slot >= 1) {
        const double dd = (double)d, F = 1.0 - (dd + 4.0) * kU;
        if (qb != ~0u && F > 0.5) {
            const double T = (double)ord2f(qb);
            if (T < 1e300) {
                const double rad = __builtin_sqrt((fmax(T, 0.0) + dd * 0x1p-140) / F) * (1.0 + 0x1p-40);
                double A = (double)dq * (1.0 - 0x1p-22) - rad, Bb = (double)dq * (1.0 + 0x1p-22) + rad;
                A -= __builtin_fabs(A) * 0x1p-50;
                Bb += __builtin_fabs(Bb) * 0x1p-50;
                fa = __double2float_rd(A);
                fb = __double2float_ru(Bb);
                const float2 ls = sp.lstat[p];
                if (ls.y < fa || ls.x > fb) live = -1;
            }
        }
    }
    if (sp.work && (q & 7) == 0) {  // the plan's work estimate (pair_record's, summed per query)
        int hits = 0;
#pragma unroll
        for (int i = 0; i < 16 / G; ++i) hits += est_on && valid && live >= 0 && !(ts[i].y < fa || ts[i].x > fb);
#pragma unroll
        for (int m = G / 2; m >= 1; m >>= 1) hits += __shfl_xor(hits, m, 64);
        const int est = sub == 0 ? (int)(((int64_t)((lsz + 255) / 256) * hits) / 16) : 0;
        const int tot = (int)wave_sum_u64((u64)(uint32_t)est);
        if (lane == 0 && tot) atomicAdd(sp.work + ((q >> 3) & 63), (unsigned)tot);
    }
    if (sub != 0 || !valid) return;
    sp.probe_live[pair] = praw >= n_lists ? praw : live;
    if (sp.cnt) {
        if (praw >= n_lists) atomicOr(sp.err, 1);
        if (live >= 0) atomicAdd(sp.cnt + xcd_id() * sp.nv + (sp.groups == 2 && slot >= 1 ? n_lists + live : live), 1);
    }
    if (live < 0) return;
    const float qnu = __double2float_ru(qnd * (1.0 + 0x1p-40));
    if (sp.QN) sp.QN[pair] = make_float4((float)s, qnu, __int_as_float((int)pair), dq);
    if (sp.QE) sp.QE[pair] = __double2float_ru(__builtin_sqrt(e) * (1.0 + 0x1p-40));
    if (sp.pqn) sp.pqn[pair] = qnu;
}

// One workgroup per query, wave w = tile w of its first probed partition.  The
// tile's 64 rows (contiguous in the row-major copy) are read 32 dims at a time,
// coalesced (lane l loads 16-B pieces of rows l/8 + 8 i), transposed through a
// per-wave LDS slab [row][33] (odd stride: conflict-free row reads), and lane r
// accumulates row r in search.cpp's order.  The 4 x 64 exact scores then meet
// in LDS, where wave 0 forms the bound.
// exact scores (search.cpp:253-269 order, as exact_score) of the 64 rows of one
// tile against one query, lane r -> row r: the rows (contiguous in the row-major
// copy) are read 32 dims at a time, coalesced (lane l loads 16-B pieces of rows
// l/8 + 8 i), and transposed through the wave's LDS slab [row][33] (odd stride:
// conflict-free row reads).  Wave-uniform; slab: 64 x 33 floats of its own.
template <int METRIC>
__device__ __forceinline__ float tile_exact(const float *qrow, const float *rows, int64_t d, float *slab, int lane) {
    float acc = 0.0f;
    const bool v4 = (d & 3) == 0;
    for (int64_t j0 = 0; j0 < d; j0 += 32) {
        const int nj = (int)min<int64_t>(32, d - j0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = (lane >> 3) + 8 * i, c = 4 * (lane & 7);
            const float *src = rows + (int64_t)r * d + j0 + c;
            float v[4];
            if (v4 && c + 4 <= nj) {
                const float4 f = *(const float4 *)src;
                v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = c + u < nj ? src[u] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) slab[r * 33 + c + u] = v[u];
        }
        const float qv = (lane & 31) < nj ? qrow[j0 + (lane & 31)] : 0.0f;
        __builtin_amdgcn_wave_barrier();
        for (int jj = 0; jj < nj; ++jj) {
            const float qj = __shfl(qv, jj, 64);
            const float xv = slab[lane * 33 + jj];
            if (METRIC == LIRA_METRIC_L2) {
                const float df = qj - xv;
                acc = acc + df * df;
            } else {
                acc = acc + qj * xv;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    return METRIC == LIRA_METRIC_L2 ? acc : -acc;
}

template <int METRIC>
__global__ __launch_bounds__(256) void k_seed(const float *Q, const int32_t *probe, int nprobe, int n_lists,
                                              const int32_t *tile_off, const int32_t *ids, const float *Xr,
                                              int64_t d, int64_t nq, int k, uint32_t *qbound) {
    __shared__ float slab_all[kSeedTiles][64 * 33];
    __shared__ float score_s[kSeedTiles][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    const int p = probe[q * nprobe];
    if (p < 0 || p >= n_lists) return;  // workgroup-uniform
    const int tile0 = tile_off[p], nt = min(kSeedTiles, tile_off[p + 1] - tile0);
    if (nt <= 0) return;
    const float sc = w < nt ? tile_exact<METRIC>(Q + q * d, Xr + (int64_t)(tile0 + w) * kTile * d, d, slab_all[w], lane)
                            : 0.0f;
    score_s[w][lane] = w < nt && ids[(tile0 + w) * kTile + lane] >= 0 && sc == sc ? sc : __builtin_inff();
    __syncthreads();
    if (w != 0) return;
    float m[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};  // 4 smallest
#pragma unroll
    for (int u = 0; u < kSeedTiles; ++u) {
        float v = score_s[u][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float lo = fminf(m[i], v), hi = fmaxf(m[i], v);
            m[i] = lo;
            v = hi;
        }
    }
    const int t = (k + 63) / 64;
    if (t > 4) return;
    const float mine = t == 1 ? m[0] : t == 2 ? m[1] : t == 3 ? m[2] : m[3];
    const uint32_t sorted = wave_sort64_u32(f2ord(mine));
    const int j = (k + t - 1) / t;
    const float B = ord2f((uint32_t)__shfl((int)sorted, j - 1, 64));
    if (lane == 0 && B < __builtin_inff()) qbound[q] = f2ord(B);
}

// The k-th smallest key of a sorted wave list, counting equal keys once when
// dedup (a vector stored in two partitions gives the same key twice: its exact
// score is the same sum); kEmptyKey if there are fewer.  Wave-uniform.
template <int R>
__device__ __forceinline__ u64 kth_distinct(const u64 (&lst)[R], int k, int dedup) {
    if (!dedup) return k <= 64 * R ? wave_list_at<R>(lst, k - 1) : kEmptyKey;
    const int lane = lane_id();
    int cnt = 0;
    u64 prev_last = kEmptyKey, res = kEmptyKey;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u64 up = shfl64(lst[r], lane == 0 ? 0 : lane - 1);
        const u64 prev = lane == 0 ? prev_last : up;
        const bool nd = lst[r] != kEmptyKey && !((r > 0 || lane > 0) && prev == lst[r]);
        const u64 bal = __ballot(nd);
        const bool hit = nd && cnt + mbcnt64(bal) == k - 1;
        const u64 hb = __ballot(hit);
        if (hb) res = shfl64(lst[r], __builtin_ctzll(hb));
        cnt += popc64(bal);
        prev_last = shfl64(lst[r], 63);
    }
    return res;
}

template <int R>
__device__ __forceinline__ void merge_batch_if(u64 (&lst)[R], u64 batch) {
    const u64 thr = wave_list_at<R>(lst, 64 * R - 1);
    if (__ballot(batch < thr)) wave_merge_batch<R>(lst, batch);
}

// MODE 0: the common call -- no per-partition lists, no k_rescan queue (rmode 0) -- compiled
// without those paths: no VGPR spills (22 spilled with them; SIFT1M mixture merge
// 73 -> 64 us); MODE 1: every call; MODE 2: MODE 0 for long rows (d >= 512): the
// exact re-check with 16 row pieces in flight instead of 8 (103 VGPRs, 4 waves per
// SIMD; GIST1M 1 k queries merge 47 -> 44 us mixture, 189 -> 174 latent; SIFT1M
// 1 250 queries 18.6 -> 19.3 us, so not for short rows)
template <int METRIC, int R, int MODE>
__global__ __launch_bounds__(256, 4) void k_smerge(SMergeArgs a) {  // (<= 128 VGPRs; 92 at MODE 0, R 1: 5 waves per SIMD)
    __shared__ uint32_t s_pend[4][64];
    // (w through readfirstlane: the query index, its row and every address derived
    // from them are wave-uniform to the compiler -- scalar loads of the row in exact_score)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t q = (int64_t)blockIdx.x * 4 + w;
    if (q >= a.nq) return;
    const int k = a.k, K2 = a.K2;
    const double dd = (double)a.d;
    const float *qrow = a.Q + q * a.d;
    // ||q|| only where the lists' error bound is recomputed on uncentred vectors
    // (centred: the per-pair norms pqn; a round trip off the merge's chain otherwise)
    double qnorm = 0.0;
    if (!a.centred) {
        double qs = 0.0;
        for (int64_t j = lane; j < a.d; j += 64) {
            const double x = (double)qrow[j];
            qs = __builtin_fma(x, x, qs);
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) qs += __builtin_bit_cast(double, shfl_xor64(__builtin_bit_cast(u64, qs), m));
        // rounded up by more than any summation-order difference to k_qstage's value
        qnorm = __builtin_sqrt(qs) * (1.0 + 0x1p-30);
    }
    const int32_t *prow = a.probe + q * a.nprobe;
    const int32_t *plv = a.plive ? a.plive + q * a.nprobe : prow;  // the pairs that have lists
    uint32_t *pend = s_pend[w];
    int64_t ncand = 0;
    unsigned long long n_rechecked = 0, n_rescans = 0;
    const int rmode = MODE == 1 ? a.rmode : 0;
    const bool per_partition = MODE == 1 ? a.per_partition != 0 : false;
    constexpr int U = MODE == 2 ? 16 : 8;
    const bool fall = rmode == 2 && a.rfall[q] != 0u;
    // lists + spills hold every key within reach: no list is re-scanned
    const bool sok = a.spill && !per_partition && a.scnt[q] <= (unsigned)a.scap;
    // a list of the query whose last slot is within its limit: only then can an
    // evicted key be needed (evicted keys lie above their list's final last key)
    bool any_over = false;

    u64 lst[R];
    int pc = 0;  // pending survivors (storage rows) in pend[0..pc)
    // Trun: the k-th smallest exact score re-checked so far (k distinct keys with
    // dedup) -- it bounds the final k-th exact score like T, and is usually far
    // tighter (T is a screened key + E), so the limits below tighten to it as the
    // re-checks come in: a candidate of exact score <= the final k-th has
    // s~ <= s_lim(final k-th, E) <= s_lim(Trun, E) (not with per-partition lists)
    float Trun = __builtin_inff();
    const bool tighten = !per_partition;
    auto reset = [&]() {
#pragma unroll
        for (int r = 0; r < R; ++r) lst[r] = kEmptyKey;
    };
    auto flush_pending = [&]() {
        if (!pc) return;
        u64 key = kEmptyKey;
        if (lane < pc) {
            const int pos = (int)pend[lane];
            key = make_key(exact_score<METRIC, U>(qrow, a.Xr, a.d, pos), a.ids[pos]);
        }
        n_rechecked += pc;
        merge_batch_if<R>(lst, key);
        pc = 0;
        if (tighten) {
            const u64 kk = kth_distinct<R>(lst, k, a.dedup);
            if (kk != kEmptyKey) Trun = fminf(Trun, key_score(kk));
        }
        __builtin_amdgcn_wave_barrier();
    };
    auto add = [&](bool take, uint32_t pos) {
        const u64 m = __ballot(take);
        const int n = popc64(m);
        if (!n) return;
        if (pc + n > 64) flush_pending();
        if (take) pend[pc + mbcnt64(m)] = pos;
        pc += n;
        __builtin_amdgcn_wave_barrier();
    };
    // the chunk's candidates, all exact (a list that may have dropped one)
    auto rescan = [&](int s, int p, int c, float T) {
        flush_pending();
        // (group 0's first chunk may be smaller than the rest: head[21] blocks)
        const bool g0 = a.groups == 2 && s == 0;
        const int bpc = g0 ? a.head[19] : a.bpc, b0 = g0 ? a.head[21] : bpc;
        const int tile0 = a.tile_off[p], ntl = a.tile_off[p + 1] - tile0;
        const int t0 = (c == 0 ? 0 : b0 + (c - 1) * bpc) * kSBT, t1 = min(ntl, t0 + (c == 0 ? b0 : bpc) * kSBT);
        for (int t = t0; t < t1; ++t) {
            const int pos = (tile0 + t) * kTile + lane;
            const int gid = a.ids[pos];
            u64 key = kEmptyKey;
            if (gid >= 0) {
                const float s = exact_score<METRIC>(qrow, a.Xr, a.d, pos);
                if (s <= T) key = make_key(s, gid);
            }
            merge_batch_if<R>(lst, key);
        }
    };
    // chunk counts are per virtual partition (plan): slot 0 is group 0
    auto vnch = [&](int s, int p) { return a.groups == 2 && s > 0 ? a.n_lists + p : p; };
    auto list_bound = [&](const u64 *src, double E) {
        const u64 kk = src[k - 1];
        return kk == kEmptyKey ? __builtin_inff() : __double2float_ru(bound_P<METRIC>((double)key_score(kk), E, dd));
    };

    // Lists lane-parallel: lane i walks list i (pair slot s, chunk c) key by
    // key while keys stay within lim -- one dependent load per round for all
    // lists at once (sorted lists: the rest is beyond lim); a list whose K2-th
    // key is within lim may have dropped a needed candidate and is re-scanned
    // exactly instead.
    auto take_lists = [&](int s_lo, int s_hi, float T) {
        // NC: the partial lists' chunk stride; NCe: the most chunks any bucket has
        // in this batch (head[20], the plan's), so no lane walks a chunk slot that
        // cannot exist
        const int NC = a.nch_max, NCe = a.head ? max(1, min(NC, a.head[20])) : NC, NL = (s_hi - s_lo) * NCe;
        for (int l0 = 0; l0 < NL; l0 += 64) {
            const int li = l0 + lane, s = s_lo + li / NCe, c = li % NCe;
            int p = -1;
            if (li < NL) {
                p = plv[s];
                if (p < 0 || p >= a.n_lists || c >= a.nch[vnch(s, p)]) p = -1;
            }
            const u64 *src = a.partial + ((q * a.nprobe + (p >= 0 ? s : 0)) * (int64_t)NC + (p >= 0 ? c : 0)) * K2;
            double lim = 0.0, E = 0.0;
            bool over = false, uns = a.unsorted != 0;
            if (p >= 0) {
                const double qn_s = a.centred ? (double)a.pqn[q * a.nprobe + s] : qnorm;
                E = a.pE ? (double)a.pE[(q * a.nprobe + s) * (int64_t)NC + c]
                         : err_E<METRIC>(qn_s, (double)a.rmax[p], dd, a.split, (double)a.dpad, a.centred);
                lim = s_lim<METRIC>((double)fminf(T, Trun), E, dd);
                const u64 last = src[K2 - 1];
                over = last != kEmptyKey && (double)key_score(last) <= lim;  // (kUnsortedMark: a NaN score)
                uns = uns || last == kUnsortedMark;  // an unmerged row buffer (k_screen_m): walk to its first empty key
            }
            // (with spill lists a full list is walked like any other; its evicted keys
            // are in the spill list, read below only if some list of the query is full)
            bool active = p >= 0 && (!over || sok) && rmode != 1;
            // four keys per round (two 16-B loads; K2 % 4 == 0, lists 32-B aligned):
            // the walk is one dependent load per round
            float Tl = fminf(T, Trun);
            for (int e0 = 0; __any(active); e0 += 4) {
                if (Trun < Tl) {  // (a flush tightened the bound: wave-uniform)
                    Tl = Trun;
                    if (p >= 0) lim = s_lim<METRIC>((double)Tl, E, dd);
                }
                u64 kv[4] = {kEmptyKey, kEmptyKey, kEmptyKey, kEmptyKey};
                if (active && e0 < K2) {
                    const ulonglong2 a0 = *(const ulonglong2 *)(src + e0), a1 = *(const ulonglong2 *)(src + e0 + 2);
                    kv[0] = a0.x;
                    kv[1] = a0.y;
                    kv[2] = a1.x;
                    kv[3] = a1.y;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    bool take = false;
                    if (active) {
                        take = kv[u] != kEmptyKey && (double)key_score(kv[u]) <= lim;
                        active = uns ? kv[u] != kEmptyKey : take;
                    }
                    add(take, (uint32_t)kv[u]);
                }
            }
            u64 ov = __ballot(over);
            any_over = any_over || ov != 0;
            if (sok) continue;  // (no re-scans)
            if (rmode == 1) {  // queue them for k_rescan
                if (ov) {
                    unsigned base = 0;
                    if (lane == 0) base = atomicAdd(a.rq_n, (unsigned)popc64(ov));
                    base = (unsigned)__shfl((int)base, 0, 64);
                    const unsigned at = base + (unsigned)mbcnt64(ov);
                    if (over) {
                        if (at < (unsigned)a.rq_cap)
                            a.rq[at] = make_int4((int)q, s, c, p);
                        else
                            a.rfall[q] = 1u;
                    }
                }
                continue;
            }
            n_rescans += popc64(ov);
            if (rmode == 2 && !fall) continue;  // k_rescan has them
            while (ov) {
                const int ln = __builtin_ctzll(ov);
                ov &= ov - 1;
                const int li2 = l0 + ln;
                rescan(s_lo + li2 / NCe, plv[s_lo + li2 / NCe], li2 % NCe, fminf(T, Trun));
            }
        }
    };

    if (per_partition) {
        for (int s = 0; s < a.nprobe; ++s) {
            const int p = prow[s];
            reset();
            if (p >= 0 && p < a.n_lists) {
                ncand += a.list_size[p];
                const double qn_s = a.centred ? (double)a.pqn[q * a.nprobe + s] : qnorm;
                const double E = err_E<METRIC>(qn_s, (double)a.rmax[p], dd, a.split, (double)a.dpad, a.centred);
                const u64 *base = a.partial + (q * a.nprobe + s) * (int64_t)a.nch_max * K2;
                float T = __builtin_inff();  // the pair's own bound: min over its chunk lists
                const int nc = a.nch[vnch(s, p)];
                const float *pe = a.pE ? a.pE + (q * a.nprobe + s) * (int64_t)a.nch_max : nullptr;
                for (int c0 = 0; c0 < nc; c0 += 64)
                    if (c0 + lane < nc)
                        T = fminf(T, list_bound(base + (int64_t)(c0 + lane) * K2, pe ? (double)pe[c0 + lane] : E));
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) T = fminf(T, __shfl_xor(T, m, 64));
                take_lists(s, s + 1, T);
                flush_pending();
            }
            const int64_t o = (q * a.nprobe + s) * (int64_t)k;
            emit_list<R>(lst, k, 0, METRIC, a.D + o, a.I + o);
        }
    } else {
        reset();
        float T = a.qbound && a.qbound[q] != ~0u ? ord2f(a.qbound[q]) : __builtin_inff();
        if (!a.qbound) {
            for (int s = 0; s < a.nprobe; ++s) {
                const int p = prow[s];
                if (p < 0 || p >= a.n_lists) continue;
                const double qn_s = a.centred ? (double)a.pqn[q * a.nprobe + s] : qnorm;
                const double E = err_E<METRIC>(qn_s, (double)a.rmax[p], dd, a.split, (double)a.dpad, a.centred);
                const u64 *base = a.partial + (q * a.nprobe + s) * (int64_t)a.nch_max * K2;
                for (int c = 0; c < a.nch[vnch(s, p)]; ++c) T = fminf(T, list_bound(base + (int64_t)c * K2, E));
            }
        }
        // (lane-parallel: a serial loop of dependent probe -> list-size loads was ~1/4 of
        // the merge's time at nprobe 8)
        {
            int64_t nc = 0;
            for (int s0 = 0; s0 < a.nprobe; s0 += 64) {
                const int s = s0 + lane;
                const int p = s < a.nprobe ? prow[s] : -1;
                if (p >= 0 && p < a.n_lists) nc += a.list_size[p];
            }
            ncand = (int64_t)wave_sum_u64((u64)nc);
        }
        take_lists(0, a.nprobe, T);
        if (rmode == 1) return;
        if (sok && any_over) {  // the spilled keys within their lists' limits
            const int ns = (int)a.scnt[q];
            const uint4 *sp = a.spill + q * (int64_t)a.scap;
            for (int i0 = 0; i0 < ns; i0 += 64) {
                bool take = false;
                uint32_t pos = 0;
                if (i0 + lane < ns) {
                    const uint4 r = sp[i0 + lane];
                    const u64 key = ((u64)r.y << 32) | r.x;
                    take = (double)key_score(key) <= s_lim<METRIC>((double)fminf(T, Trun), (double)__uint_as_float(r.z), dd);
                    pos = r.x;
                }
                add(take, pos);
            }
        }
        flush_pending();
        if (rmode == 2 && !fall) {  // k_rescan's exact survivors (all within T)
            const int nr = (int)min(a.rcnt[q], (unsigned)a.rcap);
            const u64 *rb = a.rbuf + q * (int64_t)a.rcap;
            for (int i0 = 0; i0 < nr; i0 += 64) merge_batch_if<R>(lst, i0 + lane < nr ? rb[i0 + lane] : kEmptyKey);
        }
        emit_list<R>(lst, k, a.dedup, METRIC, a.D + q * k, a.I + q * k);
    }
    if (lane == 0) {
        if (a.ncand) a.ncand[q] = ncand;
        if (a.stats) {
            atomicAdd(a.stats + 5, n_rechecked);
            if (n_rescans) atomicAdd(a.stats + 6, n_rescans);
        }
    }
}

// ---- k_rescan (LIRA_OPT_RESCAN 1): the queued chunks, all at once ----------
// One wave per (queued chunk, 64-row tile), grid-strided over a fixed grid (the
// queue length is on the device): exact scores as the merge's own re-scan
// computes them, the ones within the query's final bound T appended to its
// buffer (rbuf[q], rcap keys; past that rfall[q] sends the query back to the
// merge's own re-scan).  BIGANN-100M mixture: 1,629 re-scans of 32k-row chunks,
// one wave per query in the merge, were 21 ms of a 68 ms step.
struct RescanArgs {
    const int4 *rq;
    const unsigned *rq_n;
    const float *Q, *Xr;
    const int32_t *ids, *tile_off, *head;
    const uint32_t *qbound;
    u64 *rbuf;
    unsigned *rcnt, *rfall;
    int64_t d;
    int rq_cap, maxT, groups, bpc, rcap;
};

template <int METRIC>
__global__ __launch_bounds__(256) void k_rescan(RescanArgs a) {
    __shared__ float slab_all[4][64 * 33];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t W = (int64_t)gridDim.x * 4;
    const int64_t n = min(*a.rq_n, (unsigned)a.rq_cap), units = n * a.maxT;
    for (int64_t u = (int64_t)blockIdx.x * 4 + w; u < units; u += W) {
        const int64_t e = u / a.maxT;
        const int t = (int)(u - e * a.maxT);
        const int4 ent = a.rq[e];
        const int q = ent.x, s = ent.y, c = ent.z, p = ent.w;
        // the chunk's tiles, as the merge's re-scan maps them
        const bool g0 = a.groups == 2 && s == 0;
        const int bpc = g0 ? a.head[19] : a.bpc, b0 = g0 ? a.head[21] : bpc;
        const int tile0 = a.tile_off[p], ntl = a.tile_off[p + 1] - tile0;
        const int t0 = (c == 0 ? 0 : b0 + (c - 1) * bpc) * kSBT, t1 = min(ntl, t0 + (c == 0 ? b0 : bpc) * kSBT);
        if (t0 + t >= t1 || a.rfall[q]) continue;  // (wave-uniform)
        const float T = a.qbound[q] != ~0u ? ord2f(a.qbound[q]) : __builtin_inff();
        const int64_t tile = tile0 + t0 + t;
        const float sc = tile_exact<METRIC>(a.Q + (int64_t)q * a.d, a.Xr + tile * kTile * a.d, a.d, slab_all[w], lane);
        const int gid = a.ids[tile * kTile + lane];
        const bool take = gid >= 0 && sc <= T;
        const u64 m = __ballot(take);
        if (!m) continue;
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(a.rcnt + q, (unsigned)popc64(m));
        base = (unsigned)__shfl((int)base, 0, 64);
        if (base + (unsigned)popc64(m) > (unsigned)a.rcap) {
            if (lane == 0) a.rfall[q] = 1u;
            continue;
        }
        if (take) a.rbuf[(int64_t)q * a.rcap + base + mbcnt64(m)] = make_key(sc, gid);
    }
}

// ---- per-pair records + the partition filter (lira_bounds.hpp pair_record) ----
// One pair per G lanes (16; a whole wave for d > 256), the filter bound from
// qbound (k_seed_t's seed); the default L2 screen runs the same records inside
// k_seed_t<..., PAIRS> instead.
template <int G>
__global__ __launch_bounds__(256) void k_pairs(const float *Q, int64_t d, const int32_t *probe, int64_t npairs,
                                               int nprobe, int n_lists, const float *pivot, int centred,
                                               const float2 *lstat, const uint32_t *qbound, int32_t *probe_live,
                                               float4 *QN, float *QE, float *pqn, uint16_t *QH, int64_t dpad,
                                               const float *rmx, int32_t *cnt8, int nv, int groups, int32_t *err) {
    const int64_t pair = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
    const bool valid = pair < npairs;
    const int praw = valid ? probe[pair] : -1;
    const uint32_t qb = valid && lstat && qbound ? qbound[pair / nprobe] : ~0u;
    pair_record<G>(Q, d, pair, valid, praw, nprobe, n_lists, pivot, centred, lstat && qbound ? lstat : nullptr, qb,
                   probe_live, QN, QE, pqn, QH, dpad, nullptr, nullptr, rmx);
    // (cnt8) k_count's work: the live pair counted in its XCD's replica (as k_seed_p)
    if (cnt8 && valid && (threadIdx.x & (G - 1)) == 0) {
        if (praw >= n_lists) {
            atomicOr(err, 1);
        } else {
            const int live = probe_live[pair];  // (this lane's own store above)
            if (live >= 0)
                atomicAdd(cnt8 + xcd_id() * nv + (groups == 2 && (int)(pair % nprobe) >= 1 ? n_lists + live : live), 1);
        }
    }
}

// (stats on) what the plan's partition filter removed: pairs whose probe slot
// is valid but probe_live = -1 -> stats[1], and their candidates (list sizes:
// (query, candidate) pairs never screened) -> stats[3]
__global__ __launch_bounds__(256) void k_prune_stats(const int32_t *probe, const int32_t *plive, int64_t npairs,
                                                     int n_lists, const int32_t *list_size,
                                                     unsigned long long *stats) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int p = i < npairs ? probe[i] : -1;
    const bool cut = p >= 0 && p < n_lists && plive[i] < 0;
    const unsigned long long c = cut ? 1ull : 0ull, n = cut ? (unsigned long long)list_size[p] : 0ull;
    const unsigned long long cs = wave_sum_u64(c), ns = wave_sum_u64(n);
    if ((threadIdx.x & 63) == 0 && cs) {
        atomicAdd(stats + 1, cs);
        atomicAdd(stats + 3, ns);
    }
}

// ------------------------------------------------------------------ host side

static hipError_t launch_pairs(const float *Q, int64_t d, const int32_t *probe, int64_t npairs, int nprobe,
                               int n_lists, const float *pivot, int centred, const float2 *lstat,
                               const uint32_t *qbound, int32_t *probe_live, float4 *QN, float *QE, float *pqn,
                               uint16_t *QH, int64_t dpad, const float *rmx, hipStream_t st,
                               int32_t *cnt8 = nullptr, int nv = 0, int groups = 1, int32_t *err = nullptr) {
    const bool wide = d > 256;
    const unsigned g = (unsigned)((npairs * (wide ? 64 : 16) + 255) / 256);
    if (g == 0) return hipSuccess;
    // (one wave per query, G = 64 / nprobe lanes per pair as in k_seed_p, measured the same:
    // DEEP10M 80 vs 77 us per 10 k queries)
    if (wide)
        hipLaunchKernelGGL((k_pairs<64>), dim3(g), dim3(256), 0, st, Q, d, probe, npairs, nprobe, n_lists, pivot,
                           centred, lstat, qbound, probe_live, QN, QE, pqn, QH, dpad, rmx, cnt8, nv, groups, err);
    else
        hipLaunchKernelGGL((k_pairs<16>), dim3(g), dim3(256), 0, st, Q, d, probe, npairs, nprobe, n_lists, pivot,
                           centred, lstat, qbound, probe_live, QN, QE, pqn, QH, dpad, rmx, cnt8, nv, groups, err);
    return hipGetLastError();
}

static int cu_count_s(int device) {
    static int cached[64] = {0};
    if (device < 0 || device >= 64) return 256;
    if (!cached[device]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0)
            v = 256;
        cached[device] = v;
    }
    return cached[device];
}

// RL (list registers per half-wave, K2 = 32*RL >= k + 8), QR (queries per item)
static int screen_rl(int64_t k) { return k <= 24 ? 1 : k <= 56 ? 2 : k <= 120 ? 4 : k <= 248 ? 8 : -1; }
static int screen_qr(int rl) { return rl <= 1 ? 64 : 32; }
static int screen_smem(int qr, int rl) {
    return qr == 64 ? SSmem<64, 1>::total : rl == 2 ? SSmem<32, 2>::total : rl == 4 ? SSmem<32, 4>::total
                                                                          : SSmem<32, 8>::total;
}

struct SPlan {
    int rl = 1, qr = 64, K2 = 32, bpc = 1, bpc_near = 1, nch_max = 1, grid = 1, smem = 0, mfma = 1, split = 0;
    int bpc_near_min = 1, workers = 1;  // the plan picks group 0's chunk size in [bpc_near_min, bpc_near]
    int rs = 0;  // the wave-streaming screen k_screen_r (lira_rscreen.hip) instead of k_screen_m
    int waves = 4;  // (k_screen_r) waves per workgroup
    int near0 = 0;  // (k_screen_r, two groups) blocks in group 0's first chunk; 0: uniform chunks
    int pp = 0;  // per-pair query records (QN / QE / QH per pair, k_pairs or k_seed_t<.., PAIRS>)
                 // instead of k_qstage's per-block copy: the hi x hi k_screen_m
    int prescan = 0, rq_cap = 0, rcap = 0, maxT = 0;  // LIRA_OPT_RESCAN: k_rescan (queue / buffer sizes)
    int scap = 0;  // k_screen_r's spill records per query (0: no spill lists)
    int64_t max_qblk = 0;
    size_t off_rst, off_rq, off_rbuf, off_scnt, off_spill;
    size_t off_cnt, off_cursor, off_head, off_done, off_qoff, off_item, off_nch, off_qblk, off_itab, off_qlist, off_qt, off_qn,
        off_partial, off_qbound, off_pqn, off_pe, off_qe, off_live, off_cnt8, total;
};

static SPlan make_splan(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags) {
    SPlan pl;
    const lira_opts &op = idx->opt;
    pl.rl = screen_rl(k);
    const int xhi = op.xhi >= 0 ? op.xhi : idx->pivot != nullptr && (idx->metric == LIRA_METRIC_L2 || idx->ipc) ? 2 : 0;
    // k_screen_r (lira_rscreen.hip): the hi x hi screen on the centred split copy, L2
    // or centred IP (q.x = q.fl(x - c) + q.c), k <= 120 (RL 1: 64 queries per item;
    // RL 2, 4: 32), dpad <= 128, with the per-query seed, not PER_PARTITION
    // (RL 4: 32 rows with 4 waves, two workgroups per CU; LIRA_OPT_QR = 64: 64 rows with
    // 8 waves, one workgroup per CU -- half the candidate bytes per screened pair)
    const int rs_waves = pl.rl == 4 && op.qr == 64 ? 8 : 4;
    const int rs_qr = rscreen_qr(pl.rl, rs_waves);
    const bool rs = op.rscreen && (op.split || !idx->X) && (op.mfma || !idx->X) && op.seed && !(flags & (LIRA_SCAN_NO_SPLIT | LIRA_SCAN_PER_PARTITION)) &&
                    idx->Xb && idx->xadjc && idx->pivot && idx->lstat && rscreen_shape_ok(idx->dpad, k) && xhi == 2 &&
                    (op.qr == 0 || op.qr == rs_qr) && (idx->metric == LIRA_METRIC_L2 || idx->ipc) &&
                    // dpad > 128 (streamed A operands) only with LIRA_OPT_RSCREEN = 2: measured GIST1M
                    // (d = 960) latent scan + merge 1.21 ms against k_screen_m's 1.10, mixture even
                    (idx->dpad <= 128 || (op.rscreen == 2 && nq * nprobe * idx->dpad < (int64_t)UINT32_MAX));
    // the split-bf16 screen unless asked off (it is the only one without the fp32
    // tiles); a centred IP copy has no k_screen_m form: the fp32 tiles there
    const bool split_wanted = idx->ipc ? rs : (op.split && !(flags & LIRA_SCAN_NO_SPLIT)) || !idx->X;
    // MFMA screen up to RL 4 (k <= 120) on the split-bf16 copy (DEEP10M's k =
    // 100: 24.1 ms against 33.3 ms on the VALU screen); the fp32 MFMA form
    // (no split copy or LIRA_OPT_SPLIT = 0) only while its LDS fits 2
    // workgroups per CU (RL <= 2); without the fp32 tiles MFMA is all there is
    const int mfma_opt = idx->X ? op.mfma : 2;
    pl.mfma = mfma_opt == 2 ? pl.rl <= 4 : mfma_opt && pl.rl <= (idx->Xb && split_wanted ? 4 : 2);
    // queries per item of the MFMA screen: 64 (4 waves); 128 (8 waves, k <= 56)
    // halves the L2 -> LDS bytes per FMA but measured slower on every config
    // (SIFT1M 1.10 -> 1.25 ms mixture, 4.45 -> 4.66 ms latent; GIST, BIGANN too)
    const int qr_opt = op.qr == 128 ? 128 : 64;
    pl.qr = pl.mfma ? (pl.rl <= 2 ? qr_opt : 64) : screen_qr(pl.rl);
    // 32 queries per item at RL 4 (LIRA_OPT_QR = 32; the full split screen):
    // 2-wave workgroups whose 78 KB of LDS fit two per CU (64 queries: one).
    // Measured DEEP10M: scan 22.4 -> 44.6 ms (twice the staged bytes per
    // query; the occupancy did not pay for it), so opt-in only
    const bool qr32 = pl.mfma && pl.rl == 4 && op.qr == 32;
    if (qr32) pl.qr = 32;
    // split-bf16 MFMA screen (k_screen_m<..., SPLIT>) where the index holds Xb;
    // LIRA_OPT_SPLIT = 0 keeps the fp32 MFMA screen (which reads the fp32 tiles)
    pl.split = split_wanted && pl.mfma && idx->Xb != nullptr;
    if (qr32 && !pl.split) pl.qr = 64;  // (built for the split copy only)
    // hi-only x (LIRA_OPT_XHI): k_screen_m at 64 queries per item
    // (default: with its 3-slot ring and pipelined fragment reads, measured
    // SIFT1M scan 2.21 -> 1.93 ms latent, 0.56 -> 0.51 mixture; GIST1M 1.49 ->
    // 1.10 latent, 1.25 -> 0.85 mixture -- more exact re-checks, fewer MFMAs)
    // IP: not centred, so the hi-only bound 2^-8 |q| R is wide against the score
    // spread (DEEP10M k = 100: merge 0.3 -> 36 ms); default off there
    // hi x hi (LIRA_OPT_XHI = 2, the L2 default): k_screen_m<..., 3>, 64 queries per
    // item, RL 1 (its 32-dim slots leave room for K2 = 32 only at 2 workgroups
    // per CU), else hi-only x.  Measured against hi-only x: SIFT1M scan 1.83 ->
    // 1.44 ms latent, 0.47 -> 0.41 mixture; GIST1M 1.03 -> 0.77 latent, 0.84 ->
    // 0.67 mixture (survivors +4 %: the bound's extra ||q - qh|| R is small
    // against the score spread)
    if (pl.split && xhi && pl.qr != 32 && pl.rl <= (pl.qr == 64 ? 4 : 1)) pl.split = 2;
    if (pl.split == 2 && xhi == 2 && pl.qr == 64 && pl.rl == 1) pl.split = 3;
    // (round 3 measured a pipelined NS-slot ring screen, k_screen_s, slower on
    // every config -- DEEP10M 28.1 vs 24.9 ms; removed in round 4, git history keeps it)
    pl.K2 = 32 * pl.rl;
    // (the wide k_screen_w and wave-resident k_screen_v screens measured 0.571 /
    // 1.50 ms against 0.325 on SIFT1M: removed in round 4)
    pl.pp = pl.split == 3;
    // k_screen_r where it applies (its own preconditions on the scan's flags are in screen_topk)
    // (with or without the fp32 tiles: the seed then comes from the row-major copy
    // and the per-pair records from k_pairs -- BIGANN-100M's compact index)
    pl.rs = rs;
    pl.waves = rs ? rs_waves : 4;
    if (rs) {
        pl.mfma = 1;
        pl.split = 3;
        pl.qr = rs_qr;
        pl.pp = 1;
    }
    pl.smem = pl.rs          ? rscreen_smem(pl.rl, pl.waves)
              : !pl.mfma     ? screen_smem(pl.qr, pl.rl)
              : pl.qr == 128 ? (pl.split == 2 ? SSmem<128, 1, true, true>::total
                                : pl.rl == 1 ? SSmem<128, 1, true>::total : SSmem<128, 2, true>::total)
              : pl.split == 3 ? SSmem<64, 1, true, false, true>::total
              : pl.qr == 32  ? SSmem<32, 4, true>::total
              : pl.split == 2 ? (pl.rl == 1 ? SSmem<64, 1, true, true>::total
                                 : pl.rl == 2 ? SSmem<64, 2, true, true>::total : SSmem<64, 4, true, true>::total)
              : pl.rl == 1   ? SSmem<64, 1, true>::total
              : pl.rl == 2   ? SSmem<64, 2, true>::total
                             : SSmem<64, 4, true>::total;
    const int64_t npairs = nq * nprobe;
    pl.grid = cu_count_s(idx->device) * std::max(1, std::min(2, (160 * 1024) / pl.smem));
    if (op.debug & 32) pl.grid = cu_count_s(idx->device);  // timing experiment: one workgroup per CU
    // ~8 items per workgroup: fewer item prologues/epilogues and row lists to
    // merge than k_scan's 16 (measured: SIFT1M scan + merge 1.47 -> 1.22 ms on
    // the mixture, 4.80 -> 4.66 ms on latent data; 4 and 32 slower overall)
    const int workers = pl.grid;
    // (k_screen_r: 4.  Its waves take an item's tiles in turn and meet at the item's
    // end, so longer items balance better: measured SIFT1M latent scan 0.80 ->
    // 0.73 ms at rounds 4 with near_rounds 1, mixture 0.253 -> 0.240 ms with
    // group 0's items at half instead of a quarter of a worker's share)
    const int rounds = op.rounds > 0 ? op.rounds : pl.rs ? 4 : 8;
    const int64_t target = (int64_t)rounds * workers;
    // (LIRA_OPT_PROBES_HINT: the probe lists are mostly -1 padding, e.g. a
    // threshold selection padded to B; size the chunking for the expected pairs)
    const int64_t npairs_est = op.probes_hint > 0 ? std::min<int64_t>(npairs, nq * op.probes_hint) : npairs;
    const int64_t est_items = (npairs_est + pl.qr - 1) / pl.qr + std::min<int64_t>(idx->n_lists, npairs_est);
    const int64_t max_blocks = std::max<int64_t>(1, (idx->max_list_tiles + kSBT - 1) / kSBT);
    if (est_items >= target) {
        pl.bpc = (int)max_blocks;
    } else {
        const int64_t split = (target + est_items - 1) / std::max<int64_t>(1, est_items);
        pl.bpc = (int)std::max<int64_t>(1, (max_blocks + split - 1) / split);
    }
    // Group 0 (each query's nearest partition, where pruning leaves most of
    // the work) is cut finer: its items are the heavy ones, and ~1.5 of them
    // per workgroup left the slowest workgroup with two (LIRA_OPT_NEAR_ROUNDS;
    // measured SIFT1M mixture scan 1.08 -> 1.04 ms at 2, slower at 4 and 8:
    // more lists, more survivors)
    // (1 since round 4 for k_screen_m too, with its group-0 chunks fixed: DEEP10M scan
    // 22.2 -> 21.5 ms, merge 0.32 -> 0.26 ms; GIST1M mixture scan -2 %, latent even)
    const int near_rounds = op.near_rounds > 0 ? op.near_rounds : 1;
    {
        const int64_t est0 = std::min<int64_t>(nq, (nq + pl.qr - 1) / pl.qr + idx->n_lists);
        const int64_t split0 = std::max<int64_t>(1, ((int64_t)near_rounds * workers + est0 - 1) / std::max<int64_t>(1, est0));
        pl.bpc_near = (int)std::min<int64_t>(pl.bpc, std::max<int64_t>(1, (max_blocks + split0 - 1) / split0));
    }
    // k_screen_m stages the radius ranges of an item's first kBR blocks in LDS; a
    // longer item would read them from global memory inside the ring (whose
    // compiler-inserted waits drain it): cap the chunk at kBR blocks
    if (pl.mfma && idx->pivot && (idx->metric == LIRA_METRIC_L2 || pl.rs)) {
        pl.bpc = std::min(pl.bpc, SSmem<64, 1, true>::kBR);
        pl.bpc_near = std::min(pl.bpc_near, pl.bpc);
    }
    // LIRA_OPT_CHUNK: at most this many blocks per chunk (smaller chunks stay in an XCD's
    // L2 while the query blocks that share them stream them)
    if (op.chunk > 0) {
        pl.bpc = std::min(pl.bpc, op.chunk);
        pl.bpc_near = std::min(pl.bpc_near, pl.bpc);
    }
    // k_screen_m + k_smerge with the default near_rounds: the plan picks group 0's
    // chunk size on the device (plan_body) from the seed's estimate of the blocks
    // the batch will screen, down to 6 rounds' worth (k_screen_r: 3)
    pl.workers = (int)workers;
    pl.bpc_near_min = pl.bpc_near;
    // (screen_topk's two-group rule: group 0's chunks exist only then)
    const bool two = !(flags & LIRA_SCAN_PER_PARTITION) && op.two_phase && nprobe >= 2 &&
                     (op.two_phase == 2 || nq >= (int64_t)pl.qr * idx->n_lists ||
                      nq * nprobe >= 4 * (int64_t)pl.qr * idx->n_lists);
    // (only k_screen_r on a small batch: without the device-side choice SIFT1M
    // mixture scan 0.242 -> 0.226 ms at 10 k queries, latent unchanged, 2 % slower at
    // 1 250; k_screen_m: GIST1M mixture scan -2 %, DEEP10M scan 22.2 -> 21.5 ms and
    // merge 0.32 -> 0.26 ms)
    if (two && op.near_rounds <= 0 && pl.mfma && pl.rs && nq < 4096) {
        const int64_t est0 = std::min<int64_t>(nq, (nq + pl.qr - 1) / pl.qr + idx->n_lists);
        const int64_t split6 = std::max<int64_t>(1, ((pl.rs ? 3 : 6) * (int64_t)workers + est0 - 1) / std::max<int64_t>(1, est0));
        pl.bpc_near_min = (int)std::min<int64_t>(pl.bpc_near, std::max<int64_t>(1, (max_blocks + split6 - 1) / split6));
    }
    // (k_screen_r) group 0's small first chunks, waited for by the query block's others
    // (default 4 blocks since round 6: SIFT1M mixture scan 0.221 -> 0.219 ms, latent equal,
    // DEEP10M mixture 1.634 -> 1.600; 6 was slower on SIFT1M)
    if (pl.rs && two) {
        const int nf = op.near_first < 0 ? 4 : op.near_first;
        pl.near0 = (int)std::min<int64_t>(nf, max_blocks);
    }
    pl.nch_max = (int)((max_blocks + pl.bpc_near_min - 1) / pl.bpc_near_min) + (pl.near0 > 0 ? 1 : 0);
    pl.max_qblk = npairs / pl.qr + std::min<int64_t>(2 * idx->n_lists, npairs) + 1;
    // the merge's chunk re-scans through k_rescan: where a chunk is long enough for
    // one wave per query to be the merge's tail (BIGANN-100M: 32k rows)
    pl.maxT = std::max(pl.bpc, pl.near0) * kSBT;
    // (k_screen_r's spill lists leave it only the queries whose spill records
    // overflow: worth the find pass only where a chunk is BIGANN-long; SIFT1M's
    // 13k-row chunks paid ~7 us of merge for it)
    pl.prescan = !(flags & LIRA_SCAN_PER_PARTITION) &&
                 (op.rescan == 1 || (op.rescan < 0 && (int64_t)pl.maxT * kTile >= (pl.rs ? 32768 : 8192)));
    if (pl.prescan) {
        pl.rq_cap = (int)std::min<int64_t>(INT32_MAX / 2, 2 * nq + 4096);
        pl.rcap = (int)std::max<int64_t>(256, (4 * k + 63) / 64 * 64);
    }
    pl.scap = pl.rs && !(flags & LIRA_SCAN_PER_PARTITION) ? (op.spill < 0 ? 256 * pl.rl : op.spill) : 0;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t at = o;
        o += (bytes + 255) & ~size_t(255);
        return at;
    };
    const size_t nl = 2 * (size_t)idx->n_lists;  // up to two groups of virtual partitions
    pl.off_cnt = take(nl * 4);
    pl.off_cnt8 = take(8 * nl * 4);  // (k_seed_p) per-XCD replicas of cnt, summed by k_plan_fill
    pl.off_cursor = take(nl * 4);
    pl.off_head = take(128 * 4);  // [0..1] totals, [2..9] XCD queue counters, [10..18] queue bounds,
                                  // [19] group 0's chunk size, [20] the most chunks of a bucket,
                                  // [21] group 0's first chunk size, [64..127] the seed's work estimates
    pl.off_done = take(pl.near0 > 0 ? (size_t)(pl.max_qblk + 1) * 4 : 0);  // per query block: first chunk done
    pl.off_rst = take(pl.prescan ? (size_t)(2 * nq + 1) * 4 : 0);  // k_rescan: [rq_n, rcnt[nq], rfall[nq]]
    pl.off_scnt = take(pl.scap ? (size_t)nq * 4 : 0);
    pl.off_qoff = take((nl + 1) * 4);
    pl.off_item = take((nl + 1) * 4);
    pl.off_nch = take(nl * 4);
    pl.off_qblk = take((nl + 1) * 4);
    pl.off_itab = take((size_t)(pl.max_qblk + 1) * pl.nch_max * 16);  // items <= query blocks x chunks
    pl.off_qlist = take((size_t)npairs * 4);
    // (per-pair records: QH, the rows' hi(q - c) per pair, in the QT slot)
    pl.off_qt = take(pl.pp ? (size_t)npairs * idx->dpad * 2 : (size_t)pl.max_qblk * pl.qr * idx->dpad * 4);
    pl.off_qn = take(pl.pp ? (size_t)npairs * 16 : (size_t)pl.max_qblk * pl.qr * 16);
    pl.off_qe = take(pl.pp ? (size_t)npairs * 4 : (size_t)pl.max_qblk * pl.qr * 4);
    pl.off_live = take((size_t)npairs * 4);
    pl.off_partial = take((size_t)npairs * pl.nch_max * pl.K2 * 8);
    pl.off_qbound = take((size_t)nq * 4);
    pl.off_pqn = take((size_t)npairs * 4);
    pl.off_pe = take((size_t)npairs * pl.nch_max * 4);  // k_screen_m: the error bound of each row list
    pl.off_rq = take((size_t)pl.rq_cap * 16);
    pl.off_rbuf = take((size_t)nq * pl.rcap * 8);
    pl.off_spill = take((size_t)nq * pl.scap * 16);
    pl.total = o;
    return pl;
}

// the screen needs the fp32 tiles (VALU / fp32 MFMA) or the split copy (split
// MFMA, k <= 120); without the tiles it is the only scan there is
bool screen_supported(const lira_index *idx, int64_t k) {
    if (screen_rl(k) <= 0 || !idx->xadj || !idx->Xr || idx->n_lists > 16384 / 2) return false;
    return idx->X != nullptr || (idx->Xb != nullptr && screen_rl(k) <= 4);
}

size_t screen_workspace_size(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags) {
    return make_splan(idx, nq, nprobe, k, flags).total;
}

// the kernel a screened scan of this shape runs (lira_scan_describe)
std::string screen_describe(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags) {
    SPlan pl = make_splan(idx, nq, nprobe, k, flags);
    std::string s = pl.rs ? std::string("k_screen_r hi-x hi-q bf16 v_mfma_f32_16x16x32_bf16 (wave-streaming)")
                    : pl.mfma ? (pl.split == 3 ? "k_screen_m hi-x hi-q bf16 v_mfma_f32_16x16x32_bf16"
                                 : pl.split == 2 ? "k_screen_m hi-x split-bf16 v_mfma_f32_16x16x32_bf16"
                                 : pl.split ? "k_screen_m split-bf16 v_mfma_f32_16x16x32_bf16"
                                        : "k_screen_m fp32 v_mfma_f32_16x16x4_f32")
                            : "k_screen VALU v_pk_fma_f32";
    s += " RL=" + std::to_string(pl.rl) + " QR=" + std::to_string(pl.qr) + " K2=" + std::to_string(pl.K2) +
         (pl.rs ? " W=" + std::to_string(pl.waves) : std::string()) +
         " grid=" + std::to_string(pl.grid) + " smem=" + std::to_string(pl.smem);
    // the plan (chunking, groups, seed, spill / re-scan): a PMC record of another plan
    // does not describe this launch's traffic (bench.py matches the whole string)
    const lira_opts &o = idx->opt;
    const bool per_part = (flags & LIRA_SCAN_PER_PARTITION) != 0;
    const bool fill = nq >= (int64_t)pl.qr * idx->n_lists || nq * nprobe >= 4 * (int64_t)pl.qr * idx->n_lists;
    const int groups = !per_part && o.two_phase && nprobe >= 2 && (o.two_phase == 2 || fill) ? 2 : 1;
    const bool fused_t = pl.pp && o.seed && idx->X && idx->metric == LIRA_METRIC_L2 && k <= 32 && idx->d <= 256;
    const bool seed_r = !fused_t && pl.rs && o.seed && idx->dpad <= 128;
    const bool fused = seed_r || fused_t;
    const int seed_t = !o.seed ? 0 : seed_r && k > 32 ? 4 : fused ? (o.seed_tiles > 0 ? o.seed_tiles : nq < 4096 ? 4 : 2)
                       : idx->X && k <= 32 ? (idx->metric != LIRA_METRIC_L2 ? 2 : o.seed_tiles > 0 ? o.seed_tiles
                                                                                   : idx->d > 512 ? 1 : 2)
                       : 4;
    s += " plan: groups=" + std::to_string(groups) + " bpc=" + std::to_string(pl.bpc) +
         " near=" + std::to_string(groups == 2 ? pl.bpc_near_min : pl.bpc) + ".." +
         std::to_string(groups == 2 ? pl.bpc_near : pl.bpc) + " near0=" + std::to_string(groups == 2 ? pl.near0 : 0) +
         " seed=" + std::to_string(seed_t) + (seed_r ? "r" : fused ? "f" : "") + " spill=" + std::to_string(pl.scap) +
         " rescan=" + std::to_string(pl.prescan);
    return s;
}

template <int M, int RL, int QR>
static hipError_t launch_screen(const ScreenArgs &a, const SPlan &pl, hipStream_t st) {
    constexpr int OCC = (160 * 1024) / SSmem<QR, RL>::total >= 2 ? 2 : 1;
    static std::atomic<uint64_t> attr{0};
    constexpr int smem = SSmem<QR, RL>::total;  // (+ the kernel's small static LDS)
    hipError_t e = set_smem_attr_once(attr, (const void *)k_screen<M, RL, QR, OCC>, smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_screen<M, RL, QR, OCC>), dim3(pl.grid), dim3(kSThreads), smem, st, a);
    return hipGetLastError();
}

template <int M, int RL, int QR, int SPLIT = 0>
static hipError_t launch_screen_m(const ScreenArgs &a, const SPlan &pl, hipStream_t st) {
    typedef SSmem<QR, RL, true, SPLIT == 2, SPLIT == 3> S;
    constexpr int OCC = (160 * 1024) / S::total >= 2 ? 2 : 1;
    static std::atomic<uint64_t> attr{0};
    constexpr int smem = S::total;  // (+ the kernel's small static LDS)
    hipError_t e = set_smem_attr_once(attr, (const void *)k_screen_m<M, RL, QR, OCC, SPLIT>, smem);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_screen_m<M, RL, QR, OCC, SPLIT>), dim3(pl.grid), dim3(QR * 4), smem, st, a);
    return hipGetLastError();
}

template <int M>
static hipError_t launch_screen_rl(const ScreenArgs &a, const SPlan &pl, hipStream_t st) {
    if (pl.mfma) {
        if (pl.qr == 128 && pl.split == 2) return launch_screen_m<M, 1, 128, 2>(a, pl, st);
        if (pl.qr == 128 && pl.split)
            return pl.rl == 1 ? launch_screen_m<M, 1, 128, 1>(a, pl, st) : launch_screen_m<M, 2, 128, 1>(a, pl, st);
        if (pl.split == 3) return launch_screen_m<M, 1, 64, 3>(a, pl, st);
        if (pl.qr == 32) return launch_screen_m<M, 4, 32, 1>(a, pl, st);
        if (pl.split == 2) switch (pl.rl) {
            case 1: return launch_screen_m<M, 1, 64, 2>(a, pl, st);
            case 2: return launch_screen_m<M, 2, 64, 2>(a, pl, st);
            default: return launch_screen_m<M, 4, 64, 2>(a, pl, st);
        }
        if (pl.qr == 128) return pl.rl == 1 ? launch_screen_m<M, 1, 128>(a, pl, st) : launch_screen_m<M, 2, 128>(a, pl, st);
        if (pl.split) switch (pl.rl) {
            case 1: return launch_screen_m<M, 1, 64, 1>(a, pl, st);
            case 2: return launch_screen_m<M, 2, 64, 1>(a, pl, st);
            default: return launch_screen_m<M, 4, 64, 1>(a, pl, st);
        }
        switch (pl.rl) {
            case 1: return launch_screen_m<M, 1, 64>(a, pl, st);
            case 2: return launch_screen_m<M, 2, 64>(a, pl, st);
            default: return launch_screen_m<M, 4, 64>(a, pl, st);
        }
    }
    switch (pl.rl) {
        case 1: return launch_screen<M, 1, 64>(a, pl, st);
        case 2: return launch_screen<M, 2, 32>(a, pl, st);
        case 4: return launch_screen<M, 4, 32>(a, pl, st);
        default: return launch_screen<M, 8, 32>(a, pl, st);
    }
}

template <int M>
static void launch_smerge(int R, const SMergeArgs &m, hipStream_t st) {
    const dim3 g((unsigned)((m.nq + 3) / 4)), b(256);
    if (!m.per_partition && m.rmode == 0 && m.d >= 512) {
        switch (R) {
            case 1: hipLaunchKernelGGL((k_smerge<M, 1, 2>), g, b, 0, st, m); break;
            case 2: hipLaunchKernelGGL((k_smerge<M, 2, 2>), g, b, 0, st, m); break;
            case 4: hipLaunchKernelGGL((k_smerge<M, 4, 2>), g, b, 0, st, m); break;
            default: hipLaunchKernelGGL((k_smerge<M, 8, 2>), g, b, 0, st, m); break;
        }
        return;
    }
    if (!m.per_partition && m.rmode == 0) {
        switch (R) {
            case 1: hipLaunchKernelGGL((k_smerge<M, 1, 0>), g, b, 0, st, m); break;
            case 2: hipLaunchKernelGGL((k_smerge<M, 2, 0>), g, b, 0, st, m); break;
            case 4: hipLaunchKernelGGL((k_smerge<M, 4, 0>), g, b, 0, st, m); break;
            default: hipLaunchKernelGGL((k_smerge<M, 8, 0>), g, b, 0, st, m); break;
        }
        return;
    }
    switch (R) {
        case 1: hipLaunchKernelGGL((k_smerge<M, 1, 1>), g, b, 0, st, m); break;
        case 2: hipLaunchKernelGGL((k_smerge<M, 2, 1>), g, b, 0, st, m); break;
        case 4: hipLaunchKernelGGL((k_smerge<M, 4, 1>), g, b, 0, st, m); break;
        default: hipLaunchKernelGGL((k_smerge<M, 8, 1>), g, b, 0, st, m); break;
    }
}

// Precondition (scan_topk): screen_supported, nq > 0, nq*nprobe < 2^31, the
// merge list size Rm valid.  ev = 4 profiling events or NULLs.
int screen_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe, int64_t nprobe, int64_t k,
                unsigned flags, int Rm, float *out_D, int64_t *out_I, int64_t *out_ncand, void *ws,
                size_t ws_bytes, hipStream_t st, hipEvent_t *ev) {
    const bool dedup = (flags & LIRA_SCAN_DEDUP) != 0;
    const bool per_part = (flags & LIRA_SCAN_PER_PARTITION) != 0;
    SPlan pl = make_splan(idx, nq, nprobe, k, flags);
    if (!ws) {
        const int rc = cached_workspace(idx, pl.total, st, &ws);
        if (rc != LIRA_OK) return rc;
    } else if (ws_bytes < pl.total) {
        return fail(LIRA_EINVAL, "workspace too small: need " + std::to_string(pl.total) + " bytes");
    }
    char *w = (char *)ws;
    int32_t *cnt = (int32_t *)(w + pl.off_cnt);
    int32_t *cursor = (int32_t *)(w + pl.off_cursor);
    int32_t *head = (int32_t *)(w + pl.off_head);
    int32_t *qoff = (int32_t *)(w + pl.off_qoff);
    int32_t *item_off = (int32_t *)(w + pl.off_item);
    int32_t *nch = (int32_t *)(w + pl.off_nch);
    int32_t *qblk = (int32_t *)(w + pl.off_qblk);
    int4 *itab = (int4 *)(w + pl.off_itab);
    int32_t *qlist = (int32_t *)(w + pl.off_qlist);
    float *QT = (float *)(w + pl.off_qt);
    float4 *QN = (float4 *)(w + pl.off_qn);
    float *QE = pl.split == 3 ? (float *)(w + pl.off_qe) : nullptr;
    u64 *partial = (u64 *)(w + pl.off_partial);
    uint32_t *qbound = per_part ? nullptr : (uint32_t *)(w + pl.off_qbound);
    const int64_t npairs = nq * nprobe;

    if (ev[0]) LIRA_HIP_TRY(hipEventRecord(ev[0], st));
    LIRA_HIP_TRY(fill32_async(w, 0u, pl.off_qoff, st));  // cnt, cursor, head, done flags (not hipMemsetAsync: lira_device.hpp)
    // Two groups (every query's first probe slot -- its nearest partition, where
    // most of its top-k lives -- queued ahead of the rest) when the bound is
    // shared across a query's items: later items then start from tight bounds.
    // Also when the first slots fill few query blocks per partition (BIGANN:
    // ~10 queries per partition) but every partition still gets >= 4 blocks of
    // pairs: the nearest-slot items then stream each bucket at most ~1/4 more
    // often, and where pruning works the rest skip almost everything (measured:
    // BIGANN-100M mixture scan 66 -> 16 ms; GIST1M's 1k queries, 2 blocks per
    // partition, latent data: 3.2 -> 3.7 ms, so not there).
    // LIRA_SCAN_TWO_PHASE: 0 off, 2 always, 1 (default) this rule.
    const lira_opts &o = idx->opt;
    const int groups_env = o.two_phase;
    const bool fill = nq >= (int64_t)pl.qr * idx->n_lists || nq * nprobe >= 4 * (int64_t)pl.qr * idx->n_lists;
    const int groups = qbound && groups_env && nprobe >= 2 && (groups_env == 2 || fill) ? 2 : 1;
    const bool tri = o.prune && !(flags & LIRA_SCAN_NO_PRUNE) && pl.mfma && idx->pivot;
    const float *tri_pivot = tri ? idx->pivot : nullptr;
    // the split screen works on centred vectors where the index has them (L2)
    const bool centred = pl.split && idx->xadjc != nullptr && idx->pivot != nullptr;
    const float *cpivot = centred ? idx->pivot : nullptr;
    float *pqn = centred ? (float *)(w + pl.off_pqn) : nullptr;
    // seed bound per query (k_seed_t / k_seed) before the plan, so that
    // k_pairs can drop the pairs whose whole list lies outside the query's
    // triangle interval under it (they get no work item and no lists)
    const bool filter = qbound && tri && o.seed && idx->lstat != nullptr;
    int32_t *plive = filter || pl.pp ? (int32_t *)(w + pl.off_live) : nullptr;
    uint16_t *QH = pl.pp ? (uint16_t *)QT : nullptr;
    // the per-pair records inside the seed kernel where it is k_seed_t (L2, k <= 32)
    // (not for d > 256: one wave per query then walked d-long chains of dependent
    // loads for its nprobe pairs; k_pairs gives every pair its own 16 lanes --
    // measured GIST1M plan 0.160 -> 0.118 ms)
    // k_screen_r's path where that fused VALU seed cannot run (IP, k > 32, the compact
    // index): the screened seed on the matrix cores, fused with the records (k_seed_r,
    // lira_rscreen.hip; 4 tiles for k > 32).  Measured against k_seed_t + k_pairs:
    // DEEP10M plan 0.244 -> 0.218 ms latent, 0.224 -> 0.193 mixture, and its tighter
    // exact k-th of 256 screened keys scan 6.29 -> 6.19 / 2.91 -> 2.83 ms; where the
    // fused k_seed_t runs (SIFT1M) it stays: k_seed_r there was plan +4..6 us
    const bool fused_t = plive && qbound && o.seed && idx->X && idx->metric == LIRA_METRIC_L2 && k <= 32 && idx->d <= 256;
    const bool seed_r = !fused_t && pl.rs && plive && pl.pp && qbound && o.seed && centred && idx->tstat &&
                        idx->lstat && idx->dpad <= 128;
    const bool fused = seed_r || fused_t;
    bool seed_split = false;  // (k_seed_r without the slots 1.. records: k_pairs below)
    bool seed_counted = false;  // (k_seed_p counted the live pairs: no k_count)
    if (qbound && !fused) LIRA_HIP_TRY(fill32_async(qbound, ~0u, (size_t)nq * 4, st));
    if (seed_r) {
        RSeedArgs sr;
        sr.metric = idx->metric;
        sr.Q = q;
        sr.probe = probe;
        sr.nprobe = (int)nprobe;
        sr.n_lists = (int)idx->n_lists;
        sr.tile_off = idx->tile_off;
        sr.Xb = (const char *)idx->Xb;
        sr.xadj = idx->xadjc;
        sr.rmax = idx->rmaxc;
        sr.rmaxx = idx->rmax;
        sr.tstat = idx->tstat;
        sr.tres = idx->tres;
        sr.pivot = idx->pivot;
        sr.lstat = filter ? idx->lstat : nullptr;
        sr.probe_live = plive;
        sr.QN = QN;
        sr.QE = QE;
        sr.pqn = pqn;
        sr.QH = QH;
        const bool adapt = groups == 2 && pl.bpc_near_min < pl.bpc_near && idx->lsamp;
        sr.list_size = adapt ? idx->list_size : nullptr;
        sr.lsamp = adapt ? idx->lsamp : nullptr;
        sr.work = adapt ? (unsigned int *)head + 64 : nullptr;
        sr.qbound = qbound;
        sr.d = idx->d;
        sr.dpad = idx->dpad;
        sr.nq = nq;
        sr.k = (int)k;
        // (nprobe > 16, no work estimate: the other slots' records in k_pairs, 16 lanes per
        // pair over the whole GPU -- one wave walking 31 slots four at a time was a chain
        // of ~8 dependent pivot-row rounds per query)
        seed_split = nprobe > 16 && !adapt;
        sr.records = seed_split ? 0 : 1;
        const int nt_r = k > 32 ? 4 : o.seed_tiles > 0 ? o.seed_tiles : nq < 4096 ? 4 : 2;
        const hipError_t e = launch_seed_r(sr, nt_r, st);
        if (e != hipSuccess) return fail(LIRA_EHIP, std::string("k_seed_r launch: ") + hipGetErrorString(e));
    } else if (fused) {
        SeedPairs sp;
        sp.pivot = idx->pivot;
        sp.centred = centred ? 1 : 0;
        sp.lstat = filter ? idx->lstat : nullptr;
        sp.probe_live = plive;
        sp.QN = pl.pp ? QN : nullptr;
        sp.QE = pl.pp ? QE : nullptr;
        sp.pqn = pl.pp ? pqn : nullptr;
        sp.QH = QH;
        // (the work estimate that sizes group 0's items: only where the plan may adapt them)
        const bool adapt = groups == 2 && pl.bpc_near_min < pl.bpc_near && idx->lsamp;
        sp.list_size = adapt ? idx->list_size : nullptr;
        sp.lsamp = adapt ? idx->lsamp : nullptr;
        sp.work = adapt ? (unsigned int *)head + 64 : nullptr;
        // (256 seed rows below 4096 queries: 1 250-query step scan 0.136 -> 0.123 ms for
        // +0.008 ms of seed; at 10 k queries the seed's +0.043 ms outweighs the scan's gain)
        const int nt_f = o.seed_tiles > 0 ? o.seed_tiles : nq < 4096 ? 4 : 2;
        // every pair record in one round (k_seed_p, nprobe <= 64): G lanes per pair
        // (k_count's atomics moved into it -- each live pair ranked by an atomic on its
        // partition's counter -- measured 49 -> 70 us: same-address atomics serialise)
        const int gp = nprobe <= 4 ? 16 : nprobe <= 8 ? 8 : nprobe <= 16 ? 4 : nprobe <= 32 ? 2 : 1;
        const dim3 g4((unsigned)((nq + 3) / 4));
        if (nprobe <= 64 && sp.pivot) {
            sp.cnt = (int32_t *)(w + pl.off_cnt8);
            sp.nv = groups * (int)idx->n_lists;
            sp.err = idx->err;
            sp.groups = groups;
            seed_counted = true;
#define LIRA_SEED_P(NTV, GV)                                                                                    \
    hipLaunchKernelGGL((k_seed_p<NTV, GV>), g4, dim3(256), 0, st, q, probe, (int)nprobe, (int)idx->n_lists,     \
                       idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k, qbound, sp)
#define LIRA_SEED_PG(NTV)                                                                                       \
    switch (gp) {                                                                                               \
        case 16: LIRA_SEED_P(NTV, 16); break;                                                                   \
        case 8: LIRA_SEED_P(NTV, 8); break;                                                                     \
        case 4: LIRA_SEED_P(NTV, 4); break;                                                                     \
        case 2: LIRA_SEED_P(NTV, 2); break;                                                                     \
        default: LIRA_SEED_P(NTV, 1); break;                                                                    \
    }
            // (a grouped form -- each slot-0 list's first tiles staged in LDS once per
            // workgroup for the queries that probe it first, then the records alone -- measured
            // 50 + 21 us against 51: the workgroups' probe-column scans and the records' own
            // latency chain cost more than the tile reads it saved)
            if (nt_f == 4) {
                LIRA_SEED_PG(4)
            } else if (nt_f == 1) {
                LIRA_SEED_PG(1)
            } else {
                LIRA_SEED_PG(2)
            }
#undef LIRA_SEED_PG
#undef LIRA_SEED_P
        } else if (nt_f == 4) {
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_L2, 4, true>), g4, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k,
                               qbound, sp);
        } else if (nt_f == 1) {
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_L2, 1, true>), g4, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k,
                               qbound, sp);
        } else {
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_L2, 2, true>), g4, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k,
                               qbound, sp);
        }
        LIRA_HIP_TRY(hipGetLastError());
    } else if (qbound && o.seed && idx->X) {  // from the fp32 tiles (coalesced)
        const dim3 g((unsigned)((nq + 3) / 4));
        // (LIRA_OPT_SEED_TILES: 64 rows instead of 128 where a row is long)
        const int st_tiles = o.seed_tiles > 0 ? o.seed_tiles : idx->d > 512 ? 1 : 2;
        if (idx->metric == LIRA_METRIC_L2 && k <= 32 && st_tiles == 1)
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_L2, 1>), g, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k, qbound, SeedPairs());
        else if (idx->metric == LIRA_METRIC_L2 && k <= 32)
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_L2, 2>), g, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k, qbound, SeedPairs());
        else if (idx->metric == LIRA_METRIC_L2)
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_L2>), g, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k, qbound, SeedPairs());
        else if (k <= 32)
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_IP, 2>), g, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k, qbound, SeedPairs());
        else
            hipLaunchKernelGGL((k_seed_t<LIRA_METRIC_IP>), g, dim3(256), 0, st, q, probe, (int)nprobe,
                               (int)idx->n_lists, idx->tile_off, idx->ids, idx->X, idx->d, idx->dpad, nq, (int)k, qbound, SeedPairs());
        LIRA_HIP_TRY(hipGetLastError());
    } else if (qbound && o.seed) {  // compact index: from the row-major copy
        if (idx->metric == LIRA_METRIC_L2)
            hipLaunchKernelGGL(k_seed<LIRA_METRIC_L2>, dim3((unsigned)nq), dim3(256), 0, st, q, probe,
                               (int)nprobe, (int)idx->n_lists, idx->tile_off, idx->ids, idx->Xr, idx->d, nq,
                               (int)k, qbound);
        else
            hipLaunchKernelGGL(k_seed<LIRA_METRIC_IP>, dim3((unsigned)nq), dim3(256), 0, st, q, probe,
                               (int)nprobe, (int)idx->n_lists, idx->tile_off, idx->ids, idx->Xr, idx->d, nq,
                               (int)k, qbound);
        LIRA_HIP_TRY(hipGetLastError());
    }
    if (plive && (!fused || seed_split)) {
        // (k_pairs writes every pair's live entry: it counts them too, per XCD -- no k_count)
        LIRA_HIP_TRY(launch_pairs(q, idx->d, probe, npairs, (int)nprobe, (int)idx->n_lists, idx->pivot,
                                  idx->ipc ? 2 : centred ? 1 : 0, filter ? idx->lstat : nullptr, filter ? qbound : nullptr,
                                  plive, pl.pp ? QN : nullptr, pl.pp ? QE : nullptr, pl.pp ? pqn : nullptr, QH, idx->dpad,
                                  idx->rmax, st, (int32_t *)(w + pl.off_cnt8), groups * (int)idx->n_lists, groups,
                                  idx->err));
        seed_counted = true;
    }
    const int32_t *pprobe = plive ? plive : probe;  // the pairs that become work
    const int nvirt = groups * (int)idx->n_lists;
    LIRA_HIP_TRY(launch_plan(idx, pprobe, npairs, (int)nprobe, pl.bpc, groups == 2 ? pl.bpc_near : pl.bpc, pl.qr, groups, cnt, cursor, qoff, item_off,
                             nch, head, qlist, qblk, itab, st,
                             groups == 2 && fused && idx->lsamp ? pl.bpc_near_min : (groups == 2 ? pl.bpc_near : pl.bpc),
                             pl.workers, pl.rs ? 2 : 4, groups == 2 ? pl.near0 : 0, seed_counted ? (int32_t *)(w + pl.off_cnt8) : nullptr));
    if (!pl.pp) {
    const dim3 qgrid((unsigned)pl.max_qblk, (unsigned)((idx->dpad + 64 * kQSlabs - 1) / (64 * kQSlabs)));
    if (pl.qr == 128 && pl.split)
        hipLaunchKernelGGL((k_qstage<128, true>), qgrid, dim3(256), 0, st, q, idx->d, idx->dpad,
                           (int)nprobe, nvirt, (int)idx->n_lists, cnt, qoff, qlist, qblk, tri_pivot, cpivot, QT, QN, pqn, QE);
    else if (pl.qr == 128)
        hipLaunchKernelGGL((k_qstage<128, false>), qgrid, dim3(256), 0, st, q, idx->d, idx->dpad,
                           (int)nprobe, nvirt, (int)idx->n_lists, cnt, qoff, qlist, qblk, tri_pivot, cpivot, QT, QN, pqn, QE);
    else if (pl.qr == 32 && pl.split)
        hipLaunchKernelGGL((k_qstage<32, true>), qgrid, dim3(256), 0, st, q, idx->d, idx->dpad,
                           (int)nprobe, nvirt, (int)idx->n_lists, cnt, qoff, qlist, qblk, tri_pivot, cpivot, QT, QN, pqn, QE);
    else if (pl.qr == 64 && pl.split)
        hipLaunchKernelGGL((k_qstage<64, true>), qgrid, dim3(256), 0, st, q, idx->d, idx->dpad,
                           (int)nprobe, nvirt, (int)idx->n_lists, cnt, qoff, qlist, qblk, tri_pivot, cpivot, QT, QN, pqn, QE);
    else if (pl.qr == 64)
        hipLaunchKernelGGL((k_qstage<64, false>), qgrid, dim3(256), 0, st, q, idx->d, idx->dpad,
                           (int)nprobe, nvirt, (int)idx->n_lists, cnt, qoff, qlist, qblk, tri_pivot, cpivot, QT, QN, pqn, QE);
    else
        hipLaunchKernelGGL((k_qstage<32, false>), qgrid, dim3(256), 0, st, q, idx->d, idx->dpad,
                           (int)nprobe, nvirt, (int)idx->n_lists, cnt, qoff, qlist, qblk, tri_pivot, cpivot, QT, QN, pqn, QE);
    LIRA_HIP_TRY(hipGetLastError());
    }
    // (measured: SIFT1M mixture 1.70 -> 1.44 ms, latent +1 %)
    if (ev[1]) LIRA_HIP_TRY(hipEventRecord(ev[1], st));

    ScreenArgs a;
    a.Q = q;
    a.pivot = tri ? idx->pivot : nullptr;
    a.tstat = tri ? idx->tstat : nullptr;
    a.tres = tri && centred && (pl.split == 2 || pl.split == 3) ? idx->tres : nullptr;
    a.dbg = o.debug;
    a.share = o.share;
    a.split = pl.split;
    a.centred = centred;
    a.X = pl.split ? (const float *)idx->Xb : idx->X;
    a.xadj = centred ? idx->xadjc : idx->xadj;
    a.rmax = centred ? idx->rmaxc : idx->rmax;
    a.tile_off = idx->tile_off;
    a.cnt = cnt;
    a.item_off = item_off;
    a.qblk_off = qblk;
    a.itab = itab;
    a.head = head;
    a.QT = QT;
    a.QN = QN;
    a.QE = QE;
    a.qoff = qoff;
    a.qlist = qlist;
    a.QH = QH;
    a.qpair = pl.pp ? 1 : 0;
    a.partial = partial;
    // the lists' own error bounds (k_screen_m only; the merge otherwise takes the list-wide one)
    float *pE = pl.mfma ? (float *)(w + pl.off_pe) : nullptr;
    a.pE = pE;
    a.qbound = qbound;
    a.d = idx->d;
    a.dpad = idx->dpad;
    a.n_lists = (int)idx->n_lists;
    a.n_virt = nvirt;
    a.nprobe = (int)nprobe;
    a.k = (int)k;
    a.bpc = pl.bpc;
    a.bpc_near = groups == 2 ? pl.bpc_near : pl.bpc;
    a.nch_max = pl.nch_max;
    a.stats = idx->stats_on ? (unsigned long long *)idx->stats : nullptr;
    hipError_t e;
    bool spilled = false;
    const bool rs_go = pl.rs && plive && pl.pp && centred && qbound && pl.bpc <= 128 && pl.bpc_near <= 128;
    if (idx->ipc && pl.split && !rs_go)  // (make_splan takes the split copy of a centred IP index only for k_screen_r)
        return fail(LIRA_EHIP, "internal: centred IP split plan without k_screen_r");
    if (rs_go) {
        RArgs r;
        r.metric = idx->metric;
        r.rmaxx = idx->rmax;
        r.Xb = (const char *)idx->Xb;
        r.xadj = idx->xadjc;
        r.rmax = idx->rmaxc;
        r.tstat = tri ? idx->tstat : nullptr;
        r.tres = idx->tres;
        r.tile_off = idx->tile_off;
        r.cnt = cnt;
        r.qoff = qoff;
        r.qlist = qlist;
        r.itab = itab;
        r.head = head;
        r.QN = QN;
        r.QE = QE;
        r.QH = QH;
        r.partial = partial;
        r.pE = pE;
        r.qbound = qbound;
        r.d = idx->d;
        r.dpad = idx->dpad;
        r.n_lists = (int)idx->n_lists;
        r.n_virt = nvirt;
        r.nprobe = (int)nprobe;
        r.k = (int)k;
        r.bpc = pl.bpc;
        r.nch_max = pl.nch_max;
        // (IP: bound_P / s_lim carry no (1 +- g) factor, err_E covers the exact sum's rounding)
        const double g = idx->metric == LIRA_METRIC_L2 ? ((double)idx->d + 4.0) * 0x1p-24 : 0.0;
        r.gP = g > 0.0 ? std::nextafter((float)((1.0 + g) * (1.0 + 0x1p-50)), INFINITY) : 1.0f;
        r.invF = g > 0.0 ? std::nextafter((float)((1.0 / (1.0 - g)) * (1.0 + 0x1p-50)), INFINITY) : 1.0f;
        r.stats = a.stats;
        r.done0 = groups == 2 && pl.near0 > 0 ? (int32_t *)(w + pl.off_done) : nullptr;
        r.spill = pl.scap ? (uint4 *)(w + pl.off_spill) : nullptr;
        r.scnt = pl.scap ? (unsigned *)(w + pl.off_scnt) : nullptr;
        r.scap = pl.scap;
        spilled = r.spill != nullptr;
        e = launch_rscreen(r, pl.rl, pl.waves, pl.grid, st);
    } else {
        e = idx->metric == LIRA_METRIC_L2 ? launch_screen_rl<LIRA_METRIC_L2>(a, pl, st)
                                          : launch_screen_rl<LIRA_METRIC_IP>(a, pl, st);
    }
    if (e != hipSuccess) return fail(LIRA_EHIP, std::string("k_screen launch: ") + hipGetErrorString(e));
    if (ev[2]) LIRA_HIP_TRY(hipEventRecord(ev[2], st));
    if (a.stats && filter && npairs > 0) {
        hipLaunchKernelGGL(k_prune_stats, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, probe, plive,
                           npairs, (int)idx->n_lists, idx->list_size, a.stats);
        LIRA_HIP_TRY(hipGetLastError());
    }

    SMergeArgs m;
    m.partial = partial;
    m.pE = pE;
    m.probe = probe;
    m.plive = plive;
    m.nch = nch;
    m.list_size = idx->list_size;
    m.tile_off = idx->tile_off;
    m.ids = idx->ids;
    m.Q = q;
    m.Xr = idx->Xr;
    m.rmax = centred ? idx->rmaxc : idx->rmax;
    m.centred = centred && !idx->ipc;  // (centred IP lists always carry their pE)
    m.pqn = pqn;
    m.qbound = qbound;
    m.D = out_D;
    m.I = out_I;
    m.ncand = out_ncand;
    m.nq = nq;
    m.d = idx->d;
    m.dpad = idx->dpad;
    m.n_lists = (int)idx->n_lists;
    m.nprobe = (int)nprobe;
    m.k = (int)k;
    m.K2 = pl.K2;
    m.nch_max = pl.nch_max;
    m.bpc = pl.bpc;
    m.bpc_near = a.bpc_near;
    m.head = head;
    m.groups = groups;
    m.dedup = dedup ? 1 : 0;
    m.per_partition = per_part ? 1 : 0;
    m.stats = a.stats;
    m.split = pl.split;
    m.unsorted = 0;
    m.rmode = 0;
    m.spill = spilled ? (const uint4 *)(w + pl.off_spill) : nullptr;
    m.scnt = spilled ? (const unsigned *)(w + pl.off_scnt) : nullptr;
    m.scap = pl.scap;
    if (pl.prescan && qbound) {
        unsigned *rst = (unsigned *)(w + pl.off_rst);
        m.rq_n = rst;
        m.rcnt = rst + 1;
        m.rfall = rst + 1 + nq;
        m.rq = (int4 *)(w + pl.off_rq);
        m.rq_cap = pl.rq_cap;
        m.rbuf = (const u64 *)(w + pl.off_rbuf);
        m.rcap = pl.rcap;
        m.rmode = 1;  // queue the chunks to re-scan
        if (idx->metric == LIRA_METRIC_L2)
            launch_smerge<LIRA_METRIC_L2>(Rm, m, st);
        else
            launch_smerge<LIRA_METRIC_IP>(Rm, m, st);
        LIRA_HIP_TRY(hipGetLastError());
        RescanArgs ra;
        ra.rq = m.rq;
        ra.rq_n = m.rq_n;
        ra.Q = q;
        ra.Xr = idx->Xr;
        ra.ids = idx->ids;
        ra.tile_off = idx->tile_off;
        ra.head = head;
        ra.qbound = qbound;
        ra.rbuf = (u64 *)(w + pl.off_rbuf);
        ra.rcnt = m.rcnt;
        ra.rfall = m.rfall;
        ra.d = idx->d;
        ra.rq_cap = pl.rq_cap;
        ra.maxT = pl.maxT;
        ra.groups = groups;
        ra.bpc = pl.bpc;
        ra.rcap = pl.rcap;
        const dim3 rg((unsigned)(8 * cu_count_s(idx->device)));
        if (idx->metric == LIRA_METRIC_L2)
            hipLaunchKernelGGL(k_rescan<LIRA_METRIC_L2>, rg, dim3(256), 0, st, ra);
        else
            hipLaunchKernelGGL(k_rescan<LIRA_METRIC_IP>, rg, dim3(256), 0, st, ra);
        LIRA_HIP_TRY(hipGetLastError());
        m.rmode = 2;
    }
    if (idx->metric == LIRA_METRIC_L2)
        launch_smerge<LIRA_METRIC_L2>(Rm, m, st);
    else
        launch_smerge<LIRA_METRIC_IP>(Rm, m, st);
    LIRA_HIP_TRY(hipGetLastError());
    if (ev[3]) LIRA_HIP_TRY(hipEventRecord(ev[3], st));
    return LIRA_OK;
}

}  // namespace lira
