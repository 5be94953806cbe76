// lira_device.hpp -- device helpers shared by the gfx950 kernels:
// ordered (score, gid) keys and wave64 bitonic networks for exact top-k.
//
// Keys.  A candidate is the 64-bit key  (ord(score) << 32) | gid  where ord()
// maps fp32 to an order-preserving u32, so unsigned key order is exactly the
// canonical (score asc, gid asc) order of oracle/lira_oracle.c.  The empty key
// is ~0 (sorts last).  Scores are l2_sq (L2) or -ip (IP), as search.cpp:483-488.
//
// Lists.  A wave keeps a sorted list of N = 64*R keys in R registers per lane;
// element e = r*64 + lane.  Merging a 64-key batch costs one bitonic sort of the
// batch (21 shuffle stages) + one bitonic merge of the list (log2 N stages).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lira_hip.h"

namespace lira {

typedef unsigned long long u64;
static constexpr u64 kEmptyKey = ~0ull;
// last slot of a screen row list whose keys are NOT sorted (compact, then empty
// keys): never a real key (its row field would be 2^32 - 2), and its score
// field is a NaN, so no bound test takes it
static constexpr u64 kUnsortedMark = ~0ull - 1;
static constexpr int kWave = 64;

__device__ __forceinline__ uint32_t f2ord(float s) {
    s = s + 0.0f;  // -0 -> +0 so both zeros order as one value (== in the oracle)
    uint32_t u = __float_as_uint(s);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ u64 make_key(float score, int32_t gid) {
    return gid < 0 ? kEmptyKey : ((u64)f2ord(score) << 32) | (uint32_t)gid;
}
__device__ __forceinline__ float key_score(u64 k) { return ord2f((uint32_t)(k >> 32)); }
__device__ __forceinline__ int32_t key_gid(u64 k) { return (int32_t)(uint32_t)(k & 0xffffffffu); }

__device__ __forceinline__ u64 kmin(u64 a, u64 b) { return a < b ? a : b; }
__device__ __forceinline__ u64 kmax(u64 a, u64 b) { return a < b ? b : a; }

// lane ^ m exchange.  Inside a 16-lane DPP row it is VALU work: quad_perm for
// m = 1, 2, row_ror:8 for 8, row_shl:4 / row_shr:4 and a select for 4;
// m = 16 is one ds_swizzle (bit mode, within 32 lanes); only m = 32 takes a
// ds_bpermute.  (__shfl_xor compiled every one of them to ds_bpermute, an LDS
// round trip per step of the sorting networks.)  m is a constant after the
// callers' unrolling, so the chain folds to one form.
__device__ __forceinline__ uint32_t xor_u32(uint32_t v, int m) {
    const int x = (int)v;
    if (m == 1) return (uint32_t)__builtin_amdgcn_update_dpp(x, x, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    if (m == 2) return (uint32_t)__builtin_amdgcn_update_dpp(x, x, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    if (m == 4) {
        const int up = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xf, 0xf, false);  // row_shl:4: lane + 4
        const int dn = __builtin_amdgcn_update_dpp(x, x, 0x114, 0xf, 0xf, false);  // row_shr:4: lane - 4
        return (uint32_t)((threadIdx.x & 4) ? dn : up);
    }
    if (m == 8) return (uint32_t)__builtin_amdgcn_update_dpp(x, x, 0x128, 0xf, 0xf, false);  // row_ror:8
    if (m == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle(x, 0x401F);  // and 0x1f, xor 0x10
    return (uint32_t)__shfl_xor(x, m, 64);
}
__device__ __forceinline__ u64 shfl_xor64(u64 v, int m) {
    const uint32_t lo = xor_u32((uint32_t)v, m), hi = xor_u32((uint32_t)(v >> 32), m);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 shfl64(u64 v, int src) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl((int)lo, src, 64);
    hi = __shfl((int)hi, src, 64);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
// sum over the wave (every lane gets it)
__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += shfl_xor64(v, m);
    return v;
}
// lane l <- lane (l & 32) | (31 - (l & 31)): reversal inside each 32-lane half,
// one ds_swizzle (bit mode: and 0x1f, xor 0x1f) per dword
__device__ __forceinline__ u64 rev32_u64(u64 v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)v, 0x7C1F);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(v >> 32), 0x7C1F);
    return ((u64)hi << 32) | lo;
}

// Full ascending bitonic sort of 64 keys, one per lane.
__device__ __forceinline__ u64 wave_sort64(u64 v) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            u64 o = shfl_xor64(v, stride);
            bool lower = (lane & stride) == 0;
            bool asc = (lane & size) == 0;
            v = (lower == asc) ? kmin(v, o) : kmax(v, o);
        }
    }
    return v;
}

// Full ascending bitonic sort of 64*R keys held R per lane (element r*64+lane).
template <int R>
__device__ __forceinline__ void wave_sort(u64 (&v)[R]) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64 * R; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {  // partner in another register of the same lane
                const int rs = stride >> 6;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if ((r & rs) == 0) {
                        const bool asc = ((r * 64) & size) == 0;
                        u64 a = v[r], b = v[r | rs];
                        v[r] = asc ? kmin(a, b) : kmax(a, b);
                        v[r | rs] = asc ? kmax(a, b) : kmin(a, b);
                    }
                }
            } else {
                const bool lower = (lane & stride) == 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool asc = ((r * 64 + lane) & size) == 0;
                    u64 o = shfl_xor64(v[r], stride);
                    v[r] = (lower == asc) ? kmin(v[r], o) : kmax(v[r], o);
                }
            }
        }
    }
}

// Sort a bitonic sequence of 64*R keys ascending.
template <int R>
__device__ __forceinline__ void wave_bitonic_merge(u64 (&v)[R]) {
    const int lane = lane_id();
#pragma unroll
    for (int rs = R / 2; rs >= 1; rs >>= 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((r & rs) == 0) {
                u64 a = v[r], b = v[r | rs];
                v[r] = kmin(a, b);
                v[r | rs] = kmax(a, b);
            }
        }
    }
#pragma unroll
    for (int stride = 32; stride > 0; stride >>= 1) {
        bool lower = (lane & stride) == 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            u64 o = shfl_xor64(v[r], stride);
            v[r] = lower ? kmin(v[r], o) : kmax(v[r], o);
        }
    }
}

// list (sorted, 64*R) <- the 64*R smallest of list U batch (batch: any order).
// Half-cleaner: only the last register can change; min(list_last, reversed
// sorted batch) keeps the smallest 64 of that register U batch and leaves the
// whole list bitonic, so one merge network re-sorts it.
template <int R>
__device__ __forceinline__ void wave_merge_batch(u64 (&list)[R], u64 batch) {
    const int lane = lane_id();
    batch = wave_sort64(batch);
    u64 rev = shfl64(batch, 63 - lane);
    list[R - 1] = kmin(list[R - 1], rev);
    wave_bitonic_merge<R>(list);
}

// ---- half-wave networks: lanes 0-31 and 32-63 each hold an independent
// sequence of 32*R keys, element e = r*32 + (lane & 31).  Both halves run the
// same instructions, so two query rows are sorted/merged at once.
template <int R>
__device__ __forceinline__ void half_sort(u64 (&v)[R]) {
    const int hl = lane_id() & 31;
#pragma unroll
    for (int size = 2; size <= 32 * R; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 32) {
                const int rs = stride >> 5;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if ((r & rs) == 0) {
                        const bool asc = ((r * 32) & size) == 0;
                        u64 a = v[r], b = v[r | rs];
                        v[r] = asc ? kmin(a, b) : kmax(a, b);
                        v[r | rs] = asc ? kmax(a, b) : kmin(a, b);
                    }
                }
            } else {
                const bool lower = (hl & stride) == 0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool asc = ((r * 32 + hl) & size) == 0;
                    u64 o = shfl_xor64(v[r], stride);
                    v[r] = (lower == asc) ? kmin(v[r], o) : kmax(v[r], o);
                }
            }
        }
    }
}

template <int R>
__device__ __forceinline__ void half_bitonic_merge(u64 (&v)[R]) {
    const int hl = lane_id() & 31;
#pragma unroll
    for (int rs = R / 2; rs >= 1; rs >>= 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((r & rs) == 0) {
                u64 a = v[r], b = v[r | rs];
                v[r] = kmin(a, b);
                v[r | rs] = kmax(a, b);
            }
        }
    }
#pragma unroll
    for (int stride = 16; stride > 0; stride >>= 1) {
        const bool lower = (hl & stride) == 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            u64 o = shfl_xor64(v[r], stride);
            v[r] = lower ? kmin(v[r], o) : kmax(v[r], o);
        }
    }
}

// Per half: list (sorted, 32*R >= 64 keys) <- the 32*R smallest of list U batch,
// batch = 64 keys in any order (2 per lane).
template <int R>
__device__ __forceinline__ void half_merge_batch(u64 (&list)[R], u64 (&batch)[2]) {
    static_assert(R >= 2, "half-wave lists hold at least 64 keys");
    const int lane = lane_id();
    half_sort<2>(batch);
    (void)lane;
    const u64 rev0 = rev32_u64(batch[1]), rev1 = rev32_u64(batch[0]);
    list[R - 2] = kmin(list[R - 2], rev0);
    list[R - 1] = kmin(list[R - 1], rev1);
    half_bitonic_merge<R>(list);
}

// Per half: list (sorted, 32*R keys) <- the 32*R smallest of list U batch,
// batch = 32 keys in any order (1 per lane).
template <int R>
__device__ __forceinline__ void half_merge_batch1(u64 (&list)[R], u64 batch) {
    const int lane = lane_id();
    u64 b[1] = {batch};
    half_sort<1>(b);
    (void)lane;
    const u64 rev = rev32_u64(b[0]);
    list[R - 1] = kmin(list[R - 1], rev);
    half_bitonic_merge<R>(list);
}

// Broadcast list element e (compile-time-unknown) to the whole wave.
template <int R>
__device__ __forceinline__ u64 wave_list_at(const u64 (&list)[R], int e) {
    u64 x = list[0];
#pragma unroll
    for (int r = 1; r < R; ++r)
        if ((e >> 6) == r) x = list[r];
    return shfl64(x, e & 63);
}

// ---- split-bf16 parts (the MFMA screen's operands) ----
// fp32 -> bf16 bits, round to nearest even.  A finite value that would round
// to infinity saturates to the largest finite bf16 (0x7f7f, sign kept), so its
// lo part below stays finite and hi + lo + e = v with |e| <= 2^-16 |v| still
// holds; a NaN stays a (quiet) NaN; infinities pass through.
__device__ __forceinline__ uint32_t bf16_rne_sat(float v) {
    const uint32_t b = __float_as_uint(v);
    if ((b & 0x7fffffffu) > 0x7f800000u) return (b >> 16) | 0x40u;  // NaN
    uint32_t r = (b + 0x7fffu + ((b >> 16) & 1u)) >> 16;
    if ((r & 0x7fffu) == 0x7f80u && (b & 0x7f800000u) != 0x7f800000u) r = (r & 0x8000u) | 0x7f7fu;
    return r;
}
// the hi (hl = 0) or lo (hl = 1) bf16 part of v: v = hi + lo + e, |e| <= 2^-16 |v|
// (v - hi is exact in fp32: Sterbenz, or hi = 0)
__device__ __forceinline__ uint32_t bf16_split_part(float v, int hl) {
    const uint32_t hi = bf16_rne_sat(v);
    return hl ? bf16_rne_sat(v - __uint_as_float(hi << 16)) : hi;
}

// 64 u32 values, one per lane: ascending bitonic sort.
__device__ __forceinline__ uint32_t wave_sort64_u32(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const uint32_t o = xor_u32(v, stride);
            const bool lower = (lane & stride) == 0, asc = (lane & size) == 0;
            v = (lower == asc) ? min(v, o) : max(v, o);
        }
    }
    return v;
}

__device__ __forceinline__ int popc64(u64 m) { return __popcll(m); }
// number of set bits of m in lanes below this lane
__device__ __forceinline__ int mbcnt64(u64 m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// ---- shared by the screening kernels (k_screen_m, k_screen_r) ----
// XCD-aware work queues (k_plan): claim the next item of this workgroup's own
// XCD's queue, stealing from the others (in order) once it is empty; -1 when
// every queue is.  Thread 0 only; xq[9] (LDS) = the queue starts + end, x /
// tries the claimant's state.
__device__ __forceinline__ int xcd_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 7u);
}
// Once the claimant's queue is empty it reads all 8 claim counters at once (one
// round trip) and steals from the first queue that still has items: walking
// the queues with one atomic each in turn cost every workgroup up to 8
// serial atomic round trips at the end of the scan.  tries = 8: all empty.
__device__ __forceinline__ int claim_item(int32_t *head, const int *xq, int &x, int &tries) {
    if (tries >= 8) return -1;
    {
        const int i = xq[x] + atomicAdd(&head[2 + x], 1);
        if (i < xq[x + 1]) return i;
    }
    for (;;) {
        int c[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) c[r] = __hip_atomic_load(&head[2 + r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int pick = -1;
#pragma unroll
        for (int s = 1; s <= 8; ++s) {
            const int r = (x + s) & 7;
            if (pick < 0 && xq[r] + c[r] < xq[r + 1]) pick = r;
        }
        if (pick < 0) {
            tries = 8;
            return -1;
        }
        x = pick;
        const int i = xq[x] + atomicAdd(&head[2 + x], 1);
        if (i < xq[x + 1]) return i;
    }
}

// Inclusive prefix sum within each 16-lane group (= DPP row): 4 row_shr
// steps with zero fill, no LDS round trips (a __shfl_up chain was 4
// dependent ds_bpermutes per selection pass)
__device__ __forceinline__ int row16_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    return v;
}
// lane 15 of each 16-lane group, broadcast to the group (the group's total)
__device__ __forceinline__ int row16_total(int inc) {
    const int t0 = __builtin_amdgcn_readlane(inc, 15), t1 = __builtin_amdgcn_readlane(inc, 31);
    const int t2 = __builtin_amdgcn_readlane(inc, 47), t3 = __builtin_amdgcn_readlane(inc, 63);
    const int g = (int)(threadIdx.x & 63) >> 4;
    return g == 0 ? t0 : g == 1 ? t1 : g == 2 ? t2 : t3;
}
// Inclusive prefix sum over the wave: the rows' DPP scans plus the earlier rows' totals
__device__ __forceinline__ int wave_incl_scan(int v) {
    v = row16_incl_scan(v);
    const int t0 = __builtin_amdgcn_readlane(v, 15), t1 = __builtin_amdgcn_readlane(v, 31);
    const int t2 = __builtin_amdgcn_readlane(v, 47);
    const int g = (int)(threadIdx.x & 63) >> 4;
    return v + (g > 0 ? t0 : 0) + (g > 1 ? t1 : 0) + (g > 2 ? t2 : 0);
}
// Inclusive prefix sums of N values per thread over a workgroup of NW waves (one
// call site per workgroup, every thread): wave scans, the waves' totals through
// LDS (ws: N x NW ints), two barriers -- a Hillis-Steele scan over 1024 threads
// took 10 steps of two barriers each.  tot[i]: the workgroup's total of value i.
template <int N, int NW>
__device__ __forceinline__ void block_incl_scan(int (&v)[N], int (&tot)[N], int *ws) {
    const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = wave_incl_scan(v[i]);
    __syncthreads();  // (ws may still be read by a previous call)
    if (lane == 63)
#pragma unroll
        for (int i = 0; i < N; ++i) ws[i * NW + w] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < N; ++i) {
        int off = 0, t = 0;
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            const int x = ws[i * NW + j];
            off += j < w ? x : 0;
            t += x;
        }
        v[i] += off;
        tot[i] = t;
    }
}
// ---- per-query merge helpers (k_merge, k_smerge) ----
__device__ __forceinline__ void emit_key(u64 key, int metric, float *D, int64_t *I) {
    if (key == kEmptyKey) {
        *D = metric == LIRA_METRIC_IP ? -__builtin_inff() : __builtin_inff();
        *I = -1;
    } else {
        float s = key_score(key);
        *D = metric == LIRA_METRIC_IP ? -s : s;
        *I = key_gid(key);
    }
}

// Append the k keys of one partial list to the wave's batch, merging full batches.
template <int R>
__device__ __forceinline__ void merge_list(u64 (&lst)[R], u64 &batch, int &bc, const u64 *src,
                                           int k) {
    const int lane = lane_id();
    for (int e0 = 0; e0 < k; e0 += 64) {
        int n = min(64, k - e0);
        if (bc + n > 64) {
            u64 thr = wave_list_at<R>(lst, 64 * R - 1);
            if (__ballot(batch < thr)) wave_merge_batch<R>(lst, batch);
            batch = kEmptyKey;
            bc = 0;
        }
        if (lane >= bc && lane < bc + n) batch = src[e0 + lane - bc];
        bc += n;
    }
}

template <int R>
__device__ __forceinline__ void flush_batch(u64 (&lst)[R], u64 &batch, int &bc) {
    if (bc) {
        u64 thr = wave_list_at<R>(lst, 64 * R - 1);
        if (__ballot(batch < thr)) wave_merge_batch<R>(lst, batch);
    }
    batch = kEmptyKey;
    bc = 0;
}

// Write the first k keys of a sorted list, optionally skipping repeated keys
// (a gid replicated across probed buckets has the same key in each).
template <int R>
__device__ __forceinline__ void emit_list(const u64 (&lst)[R], int k, int dedup, int metric,
                                          float *D, int64_t *I) {
    const int lane = lane_id();
    int outpos = 0;
    u64 prev_last = kEmptyKey;
    bool have_prev = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        u64 up = shfl64(lst[r], lane == 0 ? 0 : lane - 1);
        u64 prev = lane == 0 ? prev_last : up;
        bool has_prev = lane == 0 ? have_prev : true;
        bool keep = lst[r] != kEmptyKey && !(dedup && has_prev && prev == lst[r]);
        u64 bal = __ballot(keep);
        int pos = outpos + mbcnt64(bal);
        if (keep && pos < k) emit_key(lst[r], metric, D + pos, I + pos);
        outpos += popc64(bal);
        prev_last = shfl64(lst[r], 63);
        have_prev = true;
    }
    for (int e = outpos + lane; e < k; e += 64) emit_key(kEmptyKey, metric, D + e, I + e);
}

// ---- stream-ordered fill of 32-bit words (instead of hipMemsetAsync) ----
// The search path's per-call resets (plan counters, flags, the seed bound) are a
// kernel of our own.  Round 4 saw a captured search step fault (illegal address)
// when replayed after eager calls of the same search, while its resets were
// hipMemsetAsync; since they are kernel nodes the fault has not recurred
// (test_graph_replay_after_eager_calls).  The memset is a suspect, not a shown
// cause: a one-memset capture / eager / replay repro does not fault, but it also
// lacks the library's pattern (two captured fills of different value and size
// interleaved with the plan and scan kernels on one stream) -- DESIGN.md §7.8.
// (VEC: 16-B stores, p 16-B aligned; else one 4-B store per word, any 4-B aligned p)
template <bool VEC>
static __global__ __launch_bounds__(256) void k_fill32(uint32_t *p, uint32_t v, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256 * (VEC ? 4 : 1);
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * (VEC ? 4 : 1); i < n; i += stride) {
        if (!VEC) {
            p[i] = v;
        } else if (i + 4 <= n) {
            *(uint4 *)(p + i) = make_uint4(v, v, v, v);
        } else {
            for (int64_t j = i; j < n; ++j) p[j] = v;
        }
    }
}
// bytes: a multiple of 4; p 4-B aligned (16-B stores where p is 16-B aligned, as every
// workspace offset is; a caller's buffer, e.g. lira_centroid_gemm's out_err, may not be)
static inline hipError_t fill32_async(void *p, uint32_t v, size_t bytes, hipStream_t st) {
    const int64_t n = (int64_t)(bytes / 4);
    if (n <= 0) return hipSuccess;
    const bool vec = ((uintptr_t)p & 15) == 0;
    const int64_t blocks = (n + (vec ? 1023 : 255)) / (vec ? 1024 : 256);
    const dim3 g((unsigned)(blocks < 4096 ? blocks : 4096));
    if (vec)
        hipLaunchKernelGGL(k_fill32<true>, g, dim3(256), 0, st, (uint32_t *)p, v, n);
    else
        hipLaunchKernelGGL(k_fill32<false>, g, dim3(256), 0, st, (uint32_t *)p, v, n);
    return hipGetLastError();
}

}  // namespace lira
