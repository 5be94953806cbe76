// lira_scan.hip -- batched candidate scan + exact top-k over probed buckets
// (gfx950).  Replaces search.cpp:468-514 and the per-(query, bucket) faiss
// IndexFlat*.search calls of get_cmp_recall (LIRA_smallscale.py:158-172).
//
// Schedule (partition-major).  The (query, slot) pairs of a batch are grouped
// by the bucket they probe; a work item is (bucket, block of 32 queries, chunk
// of the bucket).  A workgroup streams the chunk's 64-row d-major tiles
// through LDS once for its 32 queries, so each candidate byte read from
// HBM/L2 serves 32 query distances instead of one (search.cpp reads it once
// per query).  The kernel is therefore VALU-bound, not HBM-bound.
//
// Exactness.  Every distance is one lane's sequential fp32 sum over dims
// 0..d-1 of fl(fl(q-x)^2) (L2) or fl(q*x) (IP), with FP contraction off
// (Makefile: -ffp-contract=off), i.e. bit-identical to search.cpp:253-269.
// Top-k is exact over (score, gid) keys (lira_device.hpp).
//
// Staging.  X tiles reach LDS by LDS-DMA (global_load_lds_dwordx4) into a
// 2-deep ring: the next 16-dim chunk streams in while the current one is
// consumed, and no registers hold in-flight tile data.
//
// Selection.  Per query row the workgroup keeps its k best keys (LDS, sorted)
// and a 32-key survivor buffer.  A row's 256 candidates of a block sit in one
// half-wave (8 per lane), so selection runs from the accumulators with no
// distance tile and no barrier: a candidate whose score passes
// the row's k-th key is appended to the buffer (ballot compaction), and only
// a full buffer costs a sort + merge, a few per row per 15.6k candidates
// instead of ~23 for merge-on-every-survivor.  Lists start empty, so an
// item's first block fills them through the same path (8 merges).
//
// Kernels (one call = 5 launches + 1 memset, stream-ordered, no host sync):
//   k_count  pairs per bucket (LDS histogram, one atomic per bucket per block)
//   k_plan   offsets, chunks per bucket, work-item prefix (one workgroup)
//   k_fill   bucket -> pair lists (LDS ranks, one reservation per bucket per block)
//   k_scan   persistent; pulls work items from an atomic head
//   k_merge  per query: merge the per-(slot, chunk) top-k lists, dedup, emit
#include <algorithm>
#include <cstdlib>
#include <string>

#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

static constexpr int kQT = 32;        // queries per work item
static constexpr int kBlockTiles = 4; // tiles per candidate block
static constexpr int kCT = kBlockTiles * kTile;  // 256 candidates per block
static_assert(kCT == 256, "selection assumes 8 candidates per lane of a half-wave");
static constexpr int kScanThreads = 256;
static constexpr int kHistMax = 16384;  // buckets the LDS histograms handle
static constexpr int kPairsPerBlock = 4096;

struct ScanArgs {
    const float *Q;       // (nq, d)
    const float *X;       // [n_tiles][dpad][64]
    const int32_t *ids;   // [n_tiles*64]
    const int32_t *tile_off;
    const int32_t *cnt, *qoff, *qlist, *item_off, *nch;
    int32_t *head;        // [0] = next item, [1] = n_items
    u64 *partial;         // [pair][nch_max][k]
    uint32_t *qbound;     // [nq] f2ord(k-th score) published per query, ~0 = none; NULL = off
    int64_t d, dpad;
    int n_lists, n_virt, nprobe, k, bpc, nch_max;
    int prune;            // L2 early abandon (off: LIRA_SCAN_NO_PRUNE, or LIRA_OPT_PRUNE = 0)
    unsigned long long *stats;  // NULL, or the work counters of lira_index_set_stats
    const float *pivot;   // L2: per-list pivot (n_lists x d) and per-tile radius bounds
    const float2 *tstat;  //     for the triangle-inequality block skip; NULL = off
};

// Work is planned over "virtual partitions" v = group * n_lists + p: with two
// groups, pairs whose probe slot is < split (each query's nearest partitions)
// form group 0 and are queued first.  Group of a pair:
__device__ __forceinline__ int virt_of(int64_t pair, int p, int nprobe, int split, int groups,
                                       int n_lists) {
    return groups == 2 && (int)(pair % nprobe) >= split ? n_lists + p : p;
}

// Pairs per bucket.  With an LDS histogram each block issues one global
// atomic per touched bucket (80k pairs on 64 buckets: 128 us -> ~5 us).
// Pairs per virtual partition.
__global__ __launch_bounds__(256) void k_count(const int32_t *probe, int64_t npairs, int n_lists,
                                               int nprobe, int split, int groups, int32_t *cnt,
                                               int32_t *err) {
    extern __shared__ int32_t hist[];
    const int n_virt = groups * n_lists;
    const bool lds = n_virt <= kHistMax;
    const int64_t s = (int64_t)blockIdx.x * kPairsPerBlock;
    const int64_t e = min<int64_t>(npairs, s + kPairsPerBlock);
    if (lds) {
        for (int b = threadIdx.x; b < n_virt; b += blockDim.x) hist[b] = 0;
        __syncthreads();
    }
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        int p = probe[i];
        if (p >= n_lists) {
            atomicOr(err, 1);
            continue;
        }
        if (p < 0) continue;
        const int v = virt_of(i, p, nprobe, split, groups, n_lists);
        atomicAdd(lds ? &hist[v] : &cnt[v], 1);
    }
    if (lds) {
        __syncthreads();
        for (int b = threadIdx.x; b < n_virt; b += blockDim.x)
            if (hist[b]) atomicAdd(&cnt[b], hist[b]);
    }
}

// One workgroup of 1024 threads: exclusive scans over the buckets.
// qr = queries per work item; qblk_off (optional) = exclusive scan of the
// query blocks ceil(cnt / qr) per virtual partition.
// (blockDim.x == 1024; plan_body is also block 0's share of k_plan_fill)
// bpc_near_min < bpc_near (two groups): group 0's chunk size is chosen here, in
// [bpc_near_min, bpc_near], as about 1 / near_div of a worker's share of the
// blocks the batch will screen -- the seed's per-pair estimates on every 8th
// query, summed in head[64..127] (k_seed_t<..., PAIRS>: whole lists for slot 0, else the share
// of the list's tiles inside the triangle interval), divided by the rows per
// item.  Where pruning leaves group 0 most of the work (SIFT1M mixture: ~25
// blocks per worker), 13-block items left ~1/3 of the workers idle at the
// end; where the work is spread (latent data) the coarse chunks stay (finer
// ones cost more row lists and looser list bounds).  head[19] = the size used
// (the screen and the merge read it).
__device__ __forceinline__ void plan_body(const int32_t *cnt, const int32_t *tile_off, int n_lists, int n_virt,
                                          int bpc, int bpc_near, int qr, int32_t *qoff, int32_t *item_off,
                                          int32_t *nch, int32_t *head, int32_t *qblk_off, int4 *itab,
                                          int bpc_near_min, int workers, int near_div, int near0) {
    // (scans: wave DPP scans + one LDS exchange, block_incl_scan; the carries between
    // 1024-wide passes are workgroup-uniform registers)
    __shared__ int32_t s_a[1024], s_b[1024], s_c[1024];
    __shared__ int32_t s_ws[3 * 16], s_nchmax, s_bpc;
    if (threadIdx.x == 0) s_nchmax = 0;
    if (bpc_near_min < bpc_near && n_virt > n_lists) {
        unsigned long long w = threadIdx.x < 64 ? (unsigned)head[64 + threadIdx.x] : 0u;
        if (threadIdx.x < 64) {
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) w += shfl_xor64(w, m);
        }
        if (threadIdx.x == 0) {
            const long long per = (long long)(8ull * w / (unsigned long long)max(1, qr)) / max(1, workers);  // (1/8 sampled)
            s_bpc = (int)min<long long>(bpc_near, max<long long>(bpc_near_min, (per + near_div - 1) / near_div));
        }
        __syncthreads();
        bpc_near = s_bpc;
    }
    // near0 > 0 (two groups): group 0's first chunk is near0 blocks, the rest
    // bpc_near; head[21] = the first chunk's size (= bpc_near when uniform)
    if (threadIdx.x == 0) {
        head[19] = bpc_near;
        head[21] = near0 > 0 && n_virt > n_lists ? near0 : bpc_near;
    }
    int carry_a = 0, carry_b = 0, carry_c = 0;
    for (int base = 0; base < n_virt; base += 1024) {
        int p = base + threadIdx.x;
        int c = 0, items = 0, nqb = 0, nc = 0;
        if (p < n_virt) {
            c = cnt[p];
            const int pp = p >= n_lists ? p - n_lists : p;
            int ntl = tile_off[pp + 1] - tile_off[pp];
            int nblk = (ntl + kBlockTiles - 1) / kBlockTiles;
            const bool g0 = n_virt > n_lists && p < n_lists;
            const int b = g0 ? bpc_near : bpc;  // group 0: bpc_near
            nc = (nblk + b - 1) / b;
            if (g0 && near0 > 0) nc = nblk <= 0 ? 0 : nblk <= near0 ? 1 : 1 + (nblk - near0 + bpc_near - 1) / bpc_near;
            nch[p] = nc;
            nqb = (c + qr - 1) / qr;
            items = nqb * nc;
        }
        int v3[3] = {c, items, nqb}, t3[3];
        block_incl_scan<3, 16>(v3, t3, s_ws);
        if (p < n_virt && nc > 0) atomicMax(&s_nchmax, nc);  // (the merge's chunk slots per bucket)
        if (p < n_virt) {
            qoff[p] = carry_a + v3[0] - c;
            item_off[p] = carry_b + v3[1] - items;
            if (qblk_off) qblk_off[p] = carry_c + v3[2] - nqb;
            // (the item table is written below, in queue order)
        }
        carry_a += t3[0];
        carry_b += t3[1];
        carry_c += t3[2];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        head[20] = s_nchmax;
        qoff[n_virt] = carry_a;
        item_off[n_virt] = carry_b;
        if (qblk_off) qblk_off[n_virt] = carry_c;
        head[0] = 0;
        head[1] = carry_b;
    }
    if (!itab) return;
    // XCD-aware item queues (the screen kernels): virtual partition v belongs to
    // queue v % 8, queue r holds its partitions' items in v order (group 0, each
    // query's nearest partition, first) and chunk-major, so the query blocks
    // that stream one chunk run on one XCD back to back and share its L2.  The
    // table is written queue by queue: v' = r m + i <-> v = 8 i + r.
    // head[2 + r]: queue r's claim counter (zeroed by the caller), head[10 + r]:
    // its start, head[18]: the end of queue 7 (= the item total).
    // The entries are written by the whole workgroup, item-parallel (entry i
    // finds its partition by a binary search over the LDS prefix sums): one
    // thread per partition writing its items in turn serialised ~30 stores
    // per thread (SIFT1M: k_plan 26 -> ~8 us).
    // Two groups, k_screen_r (near0 > 0): each queue first holds chunk 0 of its group-0 partitions (every
    // query block's nearest-partition items that start the bound chain), then
    // the rest in partition order.  The ~2 items per workgroup that start at
    // once run on the seed's bound; the later group-0 chunks start from the
    // bounds the chunk-0 items published (k-th of a chunk instead of k-th of
    // 128 seed rows): the nearest partition's survivors are most of the screen's
    // selection work (SIFT1M latent: 79 % of them on 14 % of the tiles).
    // Slots per queue: m0 chunk-0 slots, then m partition slots; s_d = the
    // slot's first chunk.
    __shared__ int32_t s_g[1024], s_d[1024];
    const int m = (n_virt + 7) / 8;
    const bool two = n_virt > n_lists;
    const int m0 = two && near0 > 0 ? (n_lists + 7) / 8 : 0, M = m0 + m;  // (k_screen_r's plans only)
    carry_b = 0;
    for (int base = 0; base < 8 * M; base += 1024) {
        const int vv = base + threadIdx.x;
        const int r = vv / M, j = vv % M;
        const bool first = j < m0;  // a chunk-0 slot
        int v = vv < 8 * M ? (first ? j : j - m0) * 8 + r : n_virt;
        if (first && v >= n_lists) v = n_virt;
        int items = 0, nqb = 0, nc = 0, c0 = 0;
        if (v < n_virt) {
            nc = nch[v];
            nqb = (cnt[v] + qr - 1) / qr;
            const bool g0 = m0 > 0 && v < n_lists;  // (group 0 with its chunk-0 slots split off)
            items = first ? (nc > 0 ? nqb : 0) : g0 ? nqb * max(0, nc - 1) : nqb * nc;
            c0 = !first && g0 ? 1 : 0;
        }
        int v1[1] = {items}, t1[1];
        block_incl_scan<1, 16>(v1, t1, s_ws);
        s_b[threadIdx.x] = v1[0];
        s_a[threadIdx.x] = v;
        s_c[threadIdx.x] = nqb;
        s_d[threadIdx.x] = c0;
        s_g[threadIdx.x] = v < n_virt ? qblk_off[v] : 0;
        __syncthreads();
        const int i0 = carry_b + v1[0] - items;
        if (vv < 8 * M && j == 0) head[10 + r] = i0;
        const int total = t1[0];
        for (int i = threadIdx.x; i < total; i += 1024) {
            int lo = 0, hi = 1023;  // first slot whose inclusive prefix exceeds i
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_b[mid] > i) hi = mid; else lo = mid + 1;
            }
            const int local = i - (lo ? s_b[lo - 1] : 0), nq_b = s_c[lo];
            const int cl = local / nq_b, qb = local - cl * nq_b;
            itab[carry_b + i] = make_int4(s_a[lo], qb, s_d[lo] + cl, s_g[lo] + qb);
        }
        carry_b += total;
        __syncthreads();  // (s_* reused by the next pass)
    }
    if (threadIdx.x == 0) head[18] = carry_b;
}
__global__ __launch_bounds__(1024) void k_plan(const int32_t *cnt, const int32_t *tile_off,
                                               int n_lists, int n_virt, int bpc, int bpc_near, int qr,
                                               int32_t *qoff,
                                               int32_t *item_off, int32_t *nch, int32_t *head,
                                               int32_t *qblk_off, int4 *itab, int bpc_near_min, int workers,
                                               int near_div, int near0) {
    plan_body(cnt, tile_off, n_lists, n_virt, bpc, bpc_near, qr, qoff, item_off, nch, head, qblk_off, itab,
              bpc_near_min, workers, near_div, near0);
}

// bucket -> pair ids.  Each block reserves its slice of every bucket once
// (global atomic), then places its pairs by LDS-atomic rank.  The order inside
// a bucket's list is arbitrary; results do not depend on it.
__global__ __launch_bounds__(256) void k_fill(const int32_t *probe, int64_t npairs, int n_lists,
                                              int nprobe, int split, int groups, const int32_t *qoff,
                                              int32_t *cursor, int32_t *qlist) {
    extern __shared__ int32_t sh[];
    const int n_virt = groups * n_lists;
    const bool lds = n_virt <= kHistMax / 2;
    int32_t *hist = sh, *base = sh + (lds ? n_virt : 0);
    const int64_t s = (int64_t)blockIdx.x * kPairsPerBlock;
    const int64_t e = min<int64_t>(npairs, s + kPairsPerBlock);
    if (!lds) {
        for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
            int p = probe[i];
            if (p < 0 || p >= n_lists) continue;
            const int v = virt_of(i, p, nprobe, split, groups, n_lists);
            qlist[qoff[v] + atomicAdd(&cursor[v], 1)] = (int32_t)i;
        }
        return;
    }
    for (int b = threadIdx.x; b < n_virt; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        int p = probe[i];
        if (p >= 0 && p < n_lists) atomicAdd(&hist[virt_of(i, p, nprobe, split, groups, n_lists)], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < n_virt; b += blockDim.x) {
        base[b] = hist[b] ? qoff[b] + atomicAdd(&cursor[b], hist[b]) : 0;
        hist[b] = 0;
    }
    __syncthreads();
    for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        int p = probe[i];
        if (p < 0 || p >= n_lists) continue;
        const int v = virt_of(i, p, nprobe, split, groups, n_lists);
        qlist[base[v] + atomicAdd(&hist[v], 1)] = (int32_t)i;
    }
}

// k_plan and k_fill in one launch (n_virt <= kFuseMax): the fill needs only the
// buckets' exclusive prefix sums, which every block recomputes from cnt in LDS
// (a few scan passes over <= 2048 counts) instead of waiting on a separate
// one-block plan kernel; block 0 also runs the plan itself (item table, queue
// bounds, chunk counts) for the screen.  One launch and one dependency fewer
// on the scan's critical path.
static constexpr int kFuseMax = 2048;
__global__ __launch_bounds__(1024) void k_plan_fill(const int32_t *probe, int64_t npairs, int n_lists, int nprobe,
                                                    int groups, const int32_t *cnt, const int32_t *tile_off, int bpc,
                                                    int bpc_near, int qr, int32_t *qoff, int32_t *item_off,
                                                    int32_t *nch, int32_t *head, int32_t *qblk_off, int4 *itab,
                                                    int32_t *cursor, int32_t *qlist, int bpc_near_min,
                                                    int workers, int near_div, int near0, const int32_t *cnt8) {
    __shared__ int32_t sq[kFuseMax], hist[kFuseMax], base[kFuseMax], ws[16];
    const int n_virt = groups * n_lists, tid = threadIdx.x;
    // block 0 plans (the item table is the screen's critical path: it does nothing
    // else), blocks 1.. fill their slices of the pairs
    if (cnt8) {  // (the seed's per-XCD counts: every block sums them into base[]; block 0
                 // also writes cnt, which its plan and the screen read)
        for (int v = tid; v < n_virt; v += 1024) {
            int c = 0;
#pragma unroll
            for (int x = 0; x < 8; ++x) c += cnt8[x * n_virt + v];
            base[v] = c;
            if (blockIdx.x == 0) ((int32_t *)cnt)[v] = c;
        }
        __threadfence_block();
        __syncthreads();
    }
    if (blockIdx.x == 0) {
        plan_body(cnt, tile_off, n_lists, n_virt, bpc, bpc_near, qr, qoff, item_off, nch, head, qblk_off, itab,
                  bpc_near_min, workers, near_div, near0);
        return;
    }
    // exclusive prefix of cnt over the virtual partitions -> sq
    int carry = 0;
    for (int b0 = 0; b0 < n_virt; b0 += 1024) {
        const int v = b0 + tid < n_virt ? (cnt8 ? base[b0 + tid] : cnt[b0 + tid]) : 0;
        int x[1] = {v}, t[1];
        block_incl_scan<1, 16>(x, t, ws);
        if (b0 + tid < n_virt) sq[b0 + tid] = carry + x[0] - v;
        carry += t[0];
    }
    for (int b = tid; b < n_virt; b += 1024) hist[b] = 0;
    __syncthreads();
    // k_fill with the local offsets
    const int64_t s = (int64_t)(blockIdx.x - 1) * kPairsPerBlock;
    const int64_t e = min<int64_t>(npairs, s + kPairsPerBlock);
    for (int64_t i = s + tid; i < e; i += 1024) {
        const int p = probe[i];
        if (p >= 0 && p < n_lists) atomicAdd(&hist[virt_of(i, p, nprobe, 1, groups, n_lists)], 1);
    }
    __syncthreads();
    for (int b = tid; b < n_virt; b += 1024) {
        base[b] = hist[b] ? sq[b] + atomicAdd(&cursor[b], hist[b]) : 0;
        hist[b] = 0;
    }
    __syncthreads();
    for (int64_t i = s + tid; i < e; i += 1024) {
        const int p = probe[i];
        if (p < 0 || p >= n_lists) continue;
        const int v = virt_of(i, p, nprobe, 1, groups, n_lists);
        qlist[base[v] + atomicAdd(&hist[v], 1)] = (int32_t)i;
    }
}

// LDS carve (bytes): a 2-deep ring of X chunks (4 tiles x 16 dims, filled by
// LDS-DMA), a 2-deep ring of Q chunks, per-query survivor buffers (32 keys),
// item metadata, per-query top-k lists (k keys).
static constexpr int kDK = 16;       // dims per staged chunk
static constexpr int kBufCap = 32;   // survivor buffer per query row (1 key per lane of a half-wave)
struct ScanSmem {
    static constexpr int kXChunk = kBlockTiles * kDK * kTile * 4;  // 16 KiB
    static constexpr int kQChunk = kDK * kQT * 4;                  // 2 KiB
    static constexpr int kX = 2 * kXChunk;
    static constexpr int kQ = 2 * kQChunk;
    static constexpr int kBuf = kQT * kBufCap * 8;                 // 8 KiB
    // meta bytes: [0, 512) ints (item, pairs, buffer fill, abandon flags),
    // [512, 640) per-row thresholds, [640, 1152) per-row block-skip radii (A, B)
    // x 2 parities, [1152, 1664) per-row query-pivot distance (lo, hi) doubles
    static constexpr int kMeta = 1664;
    static int lists(int k) { return kQT * k * 8; }
    static int total(int k) { return kX + kQ + kBuf + kMeta + lists(k); }
};

typedef __attribute__((address_space(3))) void lds_void_t;

// One LDS-DMA piece: 16 B per lane from `gsrc` into LDS at lds_addr + 16*lane
// (lds_addr wave-uniform).  Inline asm, so hipcc does not treat it as an LDS
// write it must drain (vmcnt(0)) before every later ds_read; the kernel waits
// for it explicitly at the ring hand-off.  M0 is written and restored inside
// the statement (it is compiler-reserved).
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_addr)
        : "memory");
}

// Both halves of the wave merge their row's survivor buffer (n keys, per
// half) into the row's sorted k-list in LDS.  Rows without a query
// (row_ok false) merge nothing and store nothing.
template <int RL>
__device__ __forceinline__ void flush_rows(u64 *L, const u64 *buf, int n, int k, bool row_ok) {
    const int hl = lane_id() & 31;
    u64 lst[RL];
#pragma unroll
    for (int r = 0; r < RL; ++r) {
        const int e = r * 32 + hl;
        lst[r] = (row_ok && e < k) ? L[e] : kEmptyKey;
    }
    const u64 b = (row_ok && hl < n) ? buf[hl] : kEmptyKey;
    half_merge_batch1<RL>(lst, b);
    if (row_ok) {
#pragma unroll
        for (int r = 0; r < RL; ++r) {
            const int e = r * 32 + hl;
            if (e < k) L[e] = lst[r];
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// RL: half-wave list registers, 32*RL >= k.  OCC: workgroups per CU the
// register budget is built for.  FMA: LIRA_SCAN_FMA accumulation (not exact).
template <int RL, int METRIC, int OCC, bool FMA>
__global__ __launch_bounds__(kScanThreads, OCC) void k_scan(ScanArgs a) {
    const bool PRUNE = METRIC == LIRA_METRIC_L2 && a.prune;
    const bool TRI = PRUNE && a.tstat != nullptr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    typedef ScanSmem S;
    float *Xs = (float *)smem;                                   // [2][4 tiles][16 dims][64]
    float *Qs = (float *)(smem + S::kX);                         // [2][16 dims][32 queries]
    u64 *bufs = (u64 *)(smem + S::kX + S::kQ);                   // [32 rows][32]
    int *meta = (int *)(smem + S::kX + S::kQ + S::kBuf);         // [0..4) item, [8..40) pairs, [64..96) buffer fill
    u64 *lists = (u64 *)(smem + S::kX + S::kQ + S::kBuf + S::kMeta);  // [32 rows][k]
    float *thr_s = (float *)(meta + 128);                         // [32 rows] early-abandon thresholds
    float2 *tri_s = (float2 *)(meta + 160);                       // [2][32 rows] block-skip (A, B)
    double *dq_s = (double *)(meta + 288);                        // [32 rows][lo, hi] ||q - pivot||

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = tid & 31, ty = tid >> 5;  // ty = 2*wave + half
    const int k = a.k;
    const float4 *Xg = (const float4 *)a.X;
    const uint32_t xs_lds = (uint32_t)(uintptr_t)(lds_void_t *)Xs;  // LDS byte address of the ring
    const int tstride = (int)a.dpad * (kTile / 4);  // float4 per tile
    const int nchunk = (int)(a.dpad / kDK);

    for (;;) {
        if (tid == 0) {
            int item = atomicAdd(&a.head[0], 1);
            int n_items = a.head[1];
            int ok = item < n_items;
            int p = 0, qb = 0, ch = 0;
            if (ok) {
                int lo = 0, hi = a.n_virt - 1;  // last virtual partition with item_off <= item
                while (lo < hi) {
                    int mid = (lo + hi + 1) >> 1;
                    if (a.item_off[mid] <= item) lo = mid; else hi = mid - 1;
                }
                p = lo;
                int local = item - a.item_off[p];
                int nqb = (a.cnt[p] + kQT - 1) / kQT;
                ch = local / nqb;
                qb = local - ch * nqb;
            }
            meta[0] = ok;
            meta[1] = p;
            meta[2] = qb;
            meta[3] = ch;
        }
        __syncthreads();
        if (!meta[0]) break;
        // item metadata is workgroup-uniform: keep it in SGPRs
        const int v = __builtin_amdgcn_readfirstlane(meta[1]), qb = __builtin_amdgcn_readfirstlane(meta[2]),
                  ch = __builtin_amdgcn_readfirstlane(meta[3]);
        const int p = v >= a.n_lists ? v - a.n_lists : v;  // the partition itself
        const int q0 = qb * kQT;
        const int nqb_valid = min(kQT, a.cnt[v] - q0);
        if (tid < kQT) {
            meta[8 + tid] = tid < nqb_valid ? a.qlist[a.qoff[v] + q0 + tid] : -1;
            meta[64 + tid] = 0;
        }
        for (int i = tid; i < kQT * k; i += kScanThreads) lists[i] = kEmptyKey;
        __syncthreads();

        const int tile0 = __builtin_amdgcn_readfirstlane(a.tile_off[p]);
        const int ntl = __builtin_amdgcn_readfirstlane(a.tile_off[p + 1]) - tile0;
        const int tb_begin = ch * a.bpc * kBlockTiles;
        const int tb_end = min(ntl, tb_begin + a.bpc * kBlockTiles);
        // Q staging: thread stages query slot sq, dims jj, jj+1 of each chunk;
        // rows without a query stage row 0 (their results are never kept)
        const int sq = tid & 31, jj = (tid >> 5) * 2;
        const int spair = meta[8 + sq];
        const float *qrow = a.Q + (spair >= 0 ? (int64_t)(spair / a.nprobe) * a.d : 0);
        const int dlast = (int)a.d - 1;
        bool row_ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) row_ok[u] = meta[8 + ty * 4 + u] >= 0;
        // lane tx keeps the query of row ty*4 + (tx & 3) (its pruning bound slot)
        const int my_pair = meta[8 + ty * 4 + (tx & 3)];
        const int my_q = my_pair >= 0 ? my_pair / a.nprobe : -1;
        const bool row_ok_lane = my_pair >= 0;

        // Triangle-inequality block skip (L2).  For a candidate x of list p with
        // pivot c_p: ||q - x|| >= | ||q - c_p|| - ||x - c_p|| |.  The index keeps
        // per tile bounds lo <= ||x - c_p|| <= hi (k_row_stats), so a block whose
        // radius range [lo, hi] sits farther than rad_r from ||q_r - c_p|| on
        // either side cannot hold a pair scoring <= row r's threshold T_r, with
        // rad_r = sqrt((T_r + d 2^-140) / (1 - (d+4) 2^-24)): search.cpp's fp32
        // sum is >= the real squared distance times (1-2^-24)^(d+2) minus
        // underflow (every term is a rounded non-negative square), so the fp32
        // score is > T_r.  Per row: A = dq_lo - rad (rounded down), B = dq_hi +
        // rad (rounded up); skip when hi < A or lo > B for every row.
        if (TRI) {  // ||q_r - c_p|| in double for this half's 4 rows, 8 lanes per row
            const int rrow = ty * 4 + (tx >> 3), part = tx & 7;
            const int rp = meta[8 + rrow];
            double sq = 0.0;
            if (rp >= 0) {
                const float *qr = a.Q + (int64_t)(rp / a.nprobe) * a.d;
                const float *pv = a.pivot + (int64_t)p * a.d;
                for (int j = part; j < (int)a.d; j += 8) {
                    const double df = (double)qr[j] - (double)pv[j];
                    sq = __builtin_fma(df, df, sq);
                }
            }
            sq += __shfl_xor(sq, 1, 64);
            sq += __shfl_xor(sq, 2, 64);
            sq += __shfl_xor(sq, 4, 64);
            if (part == 0) {
                const double dq = __builtin_sqrt(sq), m = (double)(a.d + 8) * 0x1p-50;
                dq_s[rrow * 2] = dq * (1.0 - m);
                dq_s[rrow * 2 + 1] = dq * (1.0 + m);
            }
            __builtin_amdgcn_wave_barrier();
        }
        // Row thresholds (lane tx < 4 of each half: row ty*4 + tx): the row's
        // k-th score or the query's published bound, +inf while neither exists,
        // NaN for rows without a query.  thr_s feeds the early abandon (own
        // rows only), tri_s[par] the block skip (read by every wave: two
        // parities, so a wave refreshing the next block's never races one still
        // testing with the current block's).
        auto refresh = [&](int par) {
            const uint32_t my_bound = a.qbound && my_q >= 0
                ? __hip_atomic_load(a.qbound + my_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
            if (tx < 4) {
                const int row = ty * 4 + tx;
                const u64 t = lists[row * k + k - 1];
                float th = !row_ok_lane ? __builtin_nanf("") : t == kEmptyKey ? __builtin_inff() : key_score(t);
                if (row_ok_lane && my_bound != ~0u) th = fminf(th, ord2f(my_bound));
                thr_s[row] = th;
                if (TRI) {
                    float2 ab = make_float2(-__builtin_inff(), __builtin_inff());  // never skip
                    const double F = 1.0 - (double)(a.d + 4) * 0x1p-24;
                    if (!row_ok_lane) {
                        ab = make_float2(__builtin_inff(), -__builtin_inff());      // no query: always
                    } else if (th < __builtin_inff() && F > 0.5) {
                        const double rad = __builtin_sqrt(((double)th + (double)a.d * 0x1p-140) / F) * (1.0 + 0x1p-40);
                        double A = dq_s[row * 2] - rad, B = dq_s[row * 2 + 1] + rad;
                        A -= __builtin_fabs(A) * 0x1p-50;
                        B += __builtin_fabs(B) * 0x1p-50;
                        ab = make_float2(__double2float_rd(A), __double2float_ru(B));
                    }
                    tri_s[par * 32 + row] = ab;
                }
            }
            __builtin_amdgcn_wave_barrier();
        };
        // radius range of the block at tile tb (its tiles inside this item)
        auto block_range = [&](int tb, float &lo, float &hi) {
            const int ntv = min(kBlockTiles, tb_end - tb);
            lo = __builtin_inff();
            hi = -__builtin_inff();
            for (int i = 0; i < ntv; ++i) {
                const float2 st = a.tstat[tile0 + tb + i];
                lo = fminf(lo, st.x);
                hi = fmaxf(hi, st.y);
            }
        };
        // first block at or after t that the skip test keeps (workgroup-uniform:
        // every wave tests all 32 rows against the same LDS values)
        auto skip_from = [&](int t, int par) {
            if (TRI) {
                const float2 ab = tri_s[par * 32 + (lane & 31)];
                while (t < tb_end) {
                    float lo, hi;
                    block_range(t, lo, hi);
                    if (!__all(hi < ab.x || lo > ab.y)) break;
                    if (a.stats && tid == 0) {
                        atomicAdd(a.stats + 4, 1ull);
                        atomicAdd(a.stats + 1, (unsigned long long)(4 * nchunk));
                    }
                    t += kBlockTiles;
                }
            }
            return t;
        };
        // Cross-item pruning: a full k-list of any item of query q holds k
        // distinct ids scoring <= its k-th score, so that score bounds q's final
        // k-th; every item of q filters against the smallest one published so
        // far (a stale value is still a valid bound; ties pass, the filter is <=).
        auto publish = [&](int u) {
            if (a.qbound && row_ok[u] && tx == 0) {
                const u64 t = lists[(ty * 4 + u) * k + k - 1];
                if (t != kEmptyKey) atomicMin(a.qbound + meta[8 + ty * 4 + u] / a.nprobe, (uint32_t)(t >> 32));
            }
        };

        // Stage chunk (tb, jc) into ring slot `slot`: X by LDS-DMA (wave w moves
        // bytes [1 KiB*w, 1 KiB*(w+1)) of each tile's 4 KiB chunk; tiles past the
        // block's end re-read its last valid tile, masked later by gid -1), and
        // this thread's two Q values into registers.  Query dims past d stage 0
        // (the index pads X with zeros there).
        float pq[2];
        auto stage = [&](int tb, int jc, int slot) {
            const int ntv = min(kBlockTiles, tb_end - tb);
            const float4 *src = Xg + (int64_t)(tile0 + tb) * tstride + jc * (kTile / 4) + tid;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(
                xs_lds + (uint32_t)(slot * (kBlockTiles * kDK * kTile) + wave * 256) * 4u);
#pragma unroll
            for (int i = 0; i < kBlockTiles; ++i)
                glds16(src + min(i, ntv - 1) * tstride, dst + (uint32_t)(i * (kDK * kTile) * 4));
            // raw loads only: the pad-dim select happens at the LDS store one
            // chunk later, so nothing here waits on vmcnt (which would also
            // wait for the DMA just issued)
#pragma unroll
            for (int u = 0; u < 2; ++u) pq[u] = qrow[min(jc + jj + u, dlast)];
        };
        int slot = 0, bi = 0;  // bi: blocks processed in this item (tri_s parity)
        int tb = tb_begin;
        if (TRI) {
            refresh(1);
            __syncthreads();
            tb = skip_from(tb_begin, 1);
        }
        if (tb < tb_end) stage(tb, 0, 0);

        for (int next_tb = tb_end; tb < tb_end; tb = next_tb, ++bi) {
            // thresholds for this block (only this wave's selection changes its
            // rows' lists, so they hold for the whole block)
            refresh(bi & 1);
            float acc[4][8];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int v = 0; v < 8; ++v) acc[u][v] = 0.0f;

            // Early abandon (L2 only).  The L2 sum adds non-negative rounded
            // squares, and fp32 round-to-nearest is monotone, so every partial
            // sum is <= the final distance: once a pair's partial sum exceeds
            // its row threshold it can never be selected.  A wave whose 2048
            // pairs are all past their thresholds stops computing (wdead); when
            // all four waves are, the workgroup drops the rest of the block's
            // chunks (flags in meta[96..104), double-buffered by chunk parity).
            bool wdead = false;
            if (TRI) {  // this wave's 8 rows all skip the block: no compute
                float lo, hi;
                block_range(tb, lo, hi);
                const float2 ab = tri_s[(bi & 1) * 32 + ty * 4 + (tx & 3)];
                wdead = __all(hi < ab.x || lo > ab.y);
            }
            int c = 0, ncomp = 0;
            for (; c < nchunk; ++c) {
                float *Qc = Qs + slot * (kDK * kQT);
#pragma unroll
                for (int u = 0; u < 2; ++u) Qc[(jj + u) * kQT + sq] = c * kDK + jj + u <= dlast ? pq[u] : 0.0f;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA (asm, uncounted by hipcc) landed
                __syncthreads();  // every wave's DMA landed; every wave is done with the other slot
                // workgroup-uniform: every wave was dead after chunk c-1
                const int *fl = meta + 96 + ((c - 1) & 1) * 4;
                const bool drop = PRUNE && c > 0 && !(fl[0] | fl[1] | fl[2] | fl[3]);
                {   // stage the next chunk (this block, or the next block's first
                    // when this one ends or is dropped) into the other slot
                    int njc = (c + 1) * kDK, ntb = tb;
                    if (drop || c + 1 == nchunk) {
                        njc = 0;
                        ntb = skip_from(tb + kBlockTiles, bi & 1);
                        next_tb = ntb;
                    }
                    if (ntb < tb_end) stage(ntb, njc, slot ^ 1);
                }
                if (drop) {  // chunk c's data (in `slot`) goes unused
                    slot ^= 1;
                    break;
                }
                const float *Xc = Xs + slot * (kBlockTiles * kDK * kTile);
                const float *qp = Qc + ty * 4;
                const float *xpa = Xc + (tx >> 4) * (kDK * kTile) + (tx & 15) * 4;
                const float *xpb = xpa + 2 * (kDK * kTile);
                // software-pipelined: LDS reads of dim j+1 are in flight while dim j
                // runs as three phases of 16 independent packed ops (sub, mul, add),
                // pinned by sched_barrier so no dependent pair sits back to back
                if (!wdead) {
                ++ncomp;
                float4 q4 = *(const float4 *)qp, xa = *(const float4 *)xpa, xb = *(const float4 *)xpb;
#pragma unroll 2
                for (int j = 0; j < kDK; ++j) {
                    const float qv[4] = {q4.x, q4.y, q4.z, q4.w};
                    const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
                    // (at j = 15 this reads past the chunk, still inside the
                    // workgroup's LDS allocation; the values are never used)
                    q4 = *(const float4 *)(qp + (j + 1) * kQT);
                    xa = *(const float4 *)(xpa + (j + 1) * kTile);
                    xb = *(const float4 *)(xpb + (j + 1) * kTile);
                    if (METRIC == LIRA_METRIC_L2 && FMA) {
                        float df[4][8];
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) df[u][v] = qv[u] - xv[v];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) acc[u][v] = __builtin_fmaf(df[u][v], df[u][v], acc[u][v]);
                        __builtin_amdgcn_sched_barrier(0);
                    } else if (METRIC == LIRA_METRIC_L2) {
                        float df[4][8];
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) df[u][v] = qv[u] - xv[v];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) df[u][v] = df[u][v] * df[u][v];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) acc[u][v] = acc[u][v] + df[u][v];
                        __builtin_amdgcn_sched_barrier(0);
                    } else if (FMA) {
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) acc[u][v] = __builtin_fmaf(qv[u], xv[v], acc[u][v]);
                        __builtin_amdgcn_sched_barrier(0);
                    } else {
                        float pr[4][8];
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) pr[u][v] = qv[u] * xv[v];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int v = 0; v < 8; ++v) acc[u][v] = acc[u][v] + pr[u][v];
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if (PRUNE) {
                    const float4 t4 = *(const float4 *)&thr_s[ty * 4];
                    const float thv[4] = {t4.x, t4.y, t4.z, t4.w};
                    bool live = false;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        float m = acc[u][0];
#pragma unroll
                        for (int v = 1; v < 8; ++v) m = fminf(m, acc[u][v]);
                        live |= m <= thv[u];
                    }
                    wdead = !__any(live);
                }
                }
                if (PRUNE && lane == 0) meta[96 + (c & 1) * 4 + wave] = !wdead;
                slot ^= 1;
            }
            if (a.stats && lane == 0) {
                atomicAdd(a.stats + 0, (unsigned long long)ncomp);
                atomicAdd(a.stats + 1, (unsigned long long)nchunk);
                if (wave == 0) {
                    atomicAdd(a.stats + 2, 1ull);
                    if (c < nchunk) atomicAdd(a.stats + 3, 1ull);
                }
            }
            if (c < nchunk || wdead) continue;  // no pair of the block (c < nchunk) / wave can pass

            // this lane's candidates: c = tx*4+v (v<4) and 128+tx*4+(v-4) (loaded
            // here, not before the chunk loop, to keep 8 VGPRs free in it)
            const int ntv = min(kBlockTiles, tb_end - tb);
            int gid[8];
            {
                const int64_t base = (int64_t)(tile0 + tb) * kTile + tx * 4;
                const int4 g0 = (tx >> 4) < ntv ? *(const int4 *)&a.ids[base] : make_int4(-1, -1, -1, -1);
                const int4 g1 = 2 + (tx >> 4) < ntv ? *(const int4 *)&a.ids[base + 128] : make_int4(-1, -1, -1, -1);
                gid[0] = g0.x; gid[1] = g0.y; gid[2] = g0.z; gid[3] = g0.w;
                gid[4] = g1.x; gid[5] = g1.y; gid[6] = g1.z; gid[7] = g1.w;
            }

            // ---- selection, per wave and per half-wave, straight from registers.
            // Half h of wave w owns rows (2w+h)*4+u; lane tx holds 8 candidates of each.
            // A candidate survives when its fp32 score is <= the row's threshold:
            // the score of the row's k-th key (+inf while the list is not full,
            // NaN -- nothing passes -- for rows without a query).  A tie at the
            // threshold with a larger id is admitted and then dropped by the merge.
            // Padding candidates (gid -1: a bucket's partial last tile, tiles past
            // its end) get a score that never passes.
            {
                bool pad = false;
#pragma unroll
                for (int v = 0; v < 8; ++v) pad |= gid[v] < 0;
                if (__any(pad)) {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v < 8; ++v)
                            if (gid[v] < 0) acc[u][v] = METRIC == LIRA_METRIC_IP ? -__builtin_inff() : __builtin_inff();
                }
            }
            float thf[4];
            bool unfilled = false;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                thf[u] = thr_s[ty * 4 + u];  // refresh() at the block start (NaN: no query)
                unfilled |= thf[u] == __builtin_inff();
            }
            if (RL <= 2 && __any(unfilled)) {
                // A row whose list is not yet full (an item's first block) gets a
                // bound from the block itself: with t = RL, lane l's t-th smallest
                // score m_l, and j = ceil(k/t), the j-th smallest m_l has j*t >= k
                // real candidates at or below it, so nothing above it can be in
                // the row's top k.  Keeps the first block from pushing all 256
                // candidates through the survivor buffers.  (For k > 64 the bound
                // is loose and measured no faster, so it is off there.)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    float sv[8];
#pragma unroll
                    for (int v = 0; v < 8; ++v) {
                        const float sc = METRIC == LIRA_METRIC_IP ? -acc[u][v] : acc[u][v];
                        sv[v] = sc == sc ? sc : __builtin_inff();
                    }
                    float m;
                    if (RL == 1) {
                        m = sv[0];
#pragma unroll
                        for (int v = 1; v < 8; ++v) m = fminf(m, sv[v]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 8; ++i)
#pragma unroll
                            for (int v = 0; v + 1 < 8 - i; ++v) {
                                const float lo = fminf(sv[v], sv[v + 1]), hi = fmaxf(sv[v], sv[v + 1]);
                                sv[v] = lo;
                                sv[v + 1] = hi;
                            }
                        m = sv[RL - 1];
                    }
                    u64 mk[1] = {((u64)f2ord(m) << 32) | (uint32_t)tx};
                    half_sort<1>(mk);
                    const int j = (k + RL - 1) / RL;  // <= 32
                    const float bound = key_score(shfl64(mk[0], (lane & 32) + j - 1));
                    if (row_ok[u]) thf[u] = fminf(thf[u], bound);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int row = ty * 4 + u;
                u64 b[8], ball = 0;
#pragma unroll
                for (int v = 0; v < 8; ++v) {
                    b[v] = __ballot((METRIC == LIRA_METRIC_IP ? -acc[u][v] : acc[u][v]) <= thf[u]);
                    ball |= b[v];
                }
                if (!ball) continue;  // wave-uniform: no survivor in either half's row
                uint32_t hb[8];  // this half's survivor masks
                int pos[8], tot = 0;
#pragma unroll
                for (int v = 0; v < 8; ++v) {
                    hb[v] = (lane & 32) ? (uint32_t)(b[v] >> 32) : (uint32_t)b[v];
                    pos[v] = tot + __popc(hb[v] & ((1u << tx) - 1u));
                    tot += __popc(hb[v]);
                }
                u64 *buf = bufs + row * kBufCap;
                int bc = meta[64 + row];
                int consumed = 0;
                for (;;) {
                    const int room = kBufCap - bc;
#pragma unroll
                    for (int v = 0; v < 8; ++v) {
                        const int rel = pos[v] - consumed;
                        if (((hb[v] >> tx) & 1u) && rel >= 0 && rel < room)
                            buf[bc + rel] = make_key(METRIC == LIRA_METRIC_IP ? -acc[u][v] : acc[u][v], gid[v]);
                    }
                    const int placed = min(room, tot - consumed);
                    bc += placed;
                    consumed += placed;
                    __builtin_amdgcn_wave_barrier();
                    if (__any(bc == kBufCap)) {  // a full buffer: merge both halves' buffers
                        flush_rows<RL>(lists + row * k, buf, bc, k, row_ok[u]);
                        publish(u);
                        bc = 0;
                    }
                    if (!__any(consumed < tot)) break;
                }
                if (tx == 0) meta[64 + row] = bc;
                __builtin_amdgcn_wave_barrier();
            }
        }

        // flush the survivor buffers, emit the k best of each row
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int row = ty * 4 + u;
            const int bc = meta[64 + row];
            if (__any(bc > 0)) {
                flush_rows<RL>(lists + row * k, bufs + row * kBufCap, bc, k, row_ok[u]);
                publish(u);
            }
            const int pair = meta[8 + row];
            if (pair >= 0) {
                u64 *dst = a.partial + ((int64_t)pair * a.nch_max + ch) * k;
                for (int e = tx; e < k; e += 32) dst[e] = lists[row * k + e];
            }
        }
        __syncthreads();
    }
}

struct MergeArgs {
    const u64 *partial;
    const int32_t *probe, *nch, *list_size;
    float *D;
    int64_t *I;
    int64_t *ncand;
    int64_t nq;
    int n_lists, nprobe, k, nch_max, metric, dedup, per_partition;
};

template <int R>
__global__ __launch_bounds__(256) void k_merge(MergeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= a.nq) return;
    const int k = a.k;
    const int32_t *prow = a.probe + q * a.nprobe;
    int64_t ncand = 0;
    if (a.per_partition) {
        for (int s = 0; s < a.nprobe; ++s) {
            int p = prow[s];
            u64 lst[R];
#pragma unroll
            for (int r = 0; r < R; ++r) lst[r] = kEmptyKey;
            if (p >= 0 && p < a.n_lists) {
                ncand += a.list_size[p];
                u64 batch = kEmptyKey;
                int bc = 0;
                for (int c = 0; c < a.nch[p]; ++c)
                    merge_list<R>(lst, batch, bc,
                                  a.partial + ((q * a.nprobe + s) * (int64_t)a.nch_max + c) * k, k);
                flush_batch<R>(lst, batch, bc);
            }
            int64_t o = (q * a.nprobe + s) * (int64_t)k;
            emit_list<R>(lst, k, 0, a.metric, a.D + o, a.I + o);
        }
    } else {
        u64 lst[R];
#pragma unroll
        for (int r = 0; r < R; ++r) lst[r] = kEmptyKey;
        u64 batch = kEmptyKey;
        int bc = 0;
        for (int s = 0; s < a.nprobe; ++s) {
            int p = prow[s];
            if (p < 0 || p >= a.n_lists) continue;
            ncand += a.list_size[p];
            for (int c = 0; c < a.nch[p]; ++c)
                merge_list<R>(lst, batch, bc,
                              a.partial + ((q * a.nprobe + s) * (int64_t)a.nch_max + c) * k, k);
        }
        flush_batch<R>(lst, batch, bc);
        emit_list<R>(lst, k, a.dedup, a.metric, a.D + q * k, a.I + q * k);
    }
    if (a.ncand && lane == 0) a.ncand[q] = ncand;
}


// ------------------------------------------------------------------ host side

struct ScanPlan {
    int bpc = 1, nch_max = 1, grid = 1, smem = 0;
    size_t off_cnt, off_cursor, off_qoff, off_item, off_nch, off_head, off_qlist, off_partial, off_qbound,
        total;
};

// half-wave list registers for k, and the workgroups per CU each variant is built for
static int scan_rl(int64_t k) { return k <= 32 ? 1 : k <= 64 ? 2 : k <= 128 ? 4 : 8; }
template <int RL>
struct ScanOcc {
    static constexpr int value = RL == 1 ? 3 : RL == 8 ? 1 : 2;
};
static int scan_occ(int rl) { return rl == 1 ? 3 : rl == 8 ? 1 : 2; }

static int merge_r(int64_t kp) {
    return kp <= 64 ? 1 : kp <= 128 ? 2 : kp <= 256 ? 4 : kp <= 512 ? 8 : -1;
}

static int cu_count(int device) {
    static int cached[64] = {0};
    if (device < 0 || device >= 64) return 256;
    if (!cached[device]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
            v <= 0)
            v = 256;
        cached[device] = v;
    }
    return cached[device];
}

static ScanPlan make_plan(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k) {
    ScanPlan pl;
    const int64_t npairs = nq * nprobe;
    const int ncu = cu_count(idx->device);
    pl.smem = ScanSmem::total((int)k);
    const int occ = std::max(1, std::min(scan_occ(scan_rl(k)), (160 * 1024) / pl.smem));
    pl.grid = ncu * occ;
    // Split buckets into chunks until the persistent grid sees ~`rounds` items
    // per workgroup, so the last, partly filled round of items is a small
    // fraction of the run (the tail); LIRA_SCAN_ROUNDS overrides (tuning).
    const int rounds = idx->opt.rounds > 0 ? idx->opt.rounds : 16;
    const int64_t target = (int64_t)rounds * pl.grid;
    const int64_t est_items = (npairs + kQT - 1) / kQT + std::min<int64_t>(idx->n_lists, npairs);
    const int64_t max_blocks = std::max<int64_t>(1, (idx->max_list_tiles + kBlockTiles - 1) / kBlockTiles);
    if (est_items >= target) {
        pl.bpc = (int)max_blocks;
    } else {
        int64_t split = (target + est_items - 1) / std::max<int64_t>(1, est_items);
        pl.bpc = (int)std::max<int64_t>(1, (max_blocks + split - 1) / split);
    }
    pl.nch_max = (int)((max_blocks + pl.bpc - 1) / pl.bpc);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        size_t at = o;
        o += (bytes + 255) & ~size_t(255);
        return at;
    };
    const size_t nv = 2 * (size_t)idx->n_lists;  // virtual partitions (two groups)
    pl.off_cnt = take(nv * 4);
    pl.off_cursor = take(nv * 4);
    pl.off_head = take(16);
    pl.off_qoff = take((nv + 1) * 4);
    pl.off_item = take((nv + 1) * 4);
    pl.off_nch = take(nv * 4);
    pl.off_qlist = take((size_t)npairs * 4);
    pl.off_partial = take((size_t)npairs * pl.nch_max * (size_t)k * 8);
    pl.off_qbound = take((size_t)nq * 4);
    pl.total = o;
    return pl;
}

template <int RL, int M, bool FMA>
static hipError_t launch_scan(const ScanArgs &a, const ScanPlan &pl, hipStream_t st) {
    constexpr int OCC = ScanOcc<RL>::value;
    static std::atomic<uint64_t> attr{0};
    hipError_t e = set_smem_attr_once(attr, (const void *)k_scan<RL, M, OCC, FMA>, 160 * 1024);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan<RL, M, OCC, FMA>), dim3(pl.grid), dim3(kScanThreads), pl.smem, st, a);
    return hipGetLastError();
}

template <int M, bool FMA>
static hipError_t launch_scan_rl(int RL, const ScanArgs &a, const ScanPlan &pl, hipStream_t st) {
    return RL == 1 ? launch_scan<1, M, FMA>(a, pl, st)
           : RL == 2 ? launch_scan<2, M, FMA>(a, pl, st)
           : RL == 4 ? launch_scan<4, M, FMA>(a, pl, st) : launch_scan<8, M, FMA>(a, pl, st);
}

template <int R>
static void launch_merge(const MergeArgs &a, hipStream_t st) {
    hipLaunchKernelGGL((k_merge<R>), dim3((unsigned)((a.nq + 3) / 4)), dim3(256), 0, st, a);
}

bool screen_supported(const lira_index *idx, int64_t k);
size_t screen_workspace_size(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags);
int screen_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe, int64_t nprobe, int64_t k,
                unsigned flags, int Rm, float *out_D, int64_t *out_I, int64_t *out_ncand, void *ws,
                size_t ws_bytes, hipStream_t st, hipEvent_t *ev);

// the screened scan (lira_screen.hip) is the default; LIRA_SCAN_EXACT,
// LIRA_SCAN_FMA or LIRA_OPT_SCREEN = 0 select the all-exact k_scan (which
// reads the fp32 tiles: LIRA_OPT_KEEP_TILES)
static bool use_screen(const lira_index *idx, int64_t k, unsigned flags) {
    return (idx->opt.screen || !idx->X) && !(flags & (LIRA_SCAN_FMA | LIRA_SCAN_EXACT)) && screen_supported(idx, k);
}

int scan_workspace_size(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags,
                        size_t *bytes) {
    ScanPlan pl = make_plan(idx, nq, nprobe, k);
    *bytes = std::max(pl.total, screen_supported(idx, k) ? screen_workspace_size(idx, nq, nprobe, k, flags) : 0);
    return LIRA_OK;
}

static int exact_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe, int64_t nprobe,
                      int64_t k, unsigned flags, int Rm, float *out_D, int64_t *out_I, int64_t *out_ncand,
                      void *ws, size_t ws_bytes, hipStream_t st, hipEvent_t *ev) {
    const bool dedup = (flags & LIRA_SCAN_DEDUP) != 0;
    const bool per_part = (flags & LIRA_SCAN_PER_PARTITION) != 0;
    const int RL = scan_rl(k);
    ScanPlan pl = make_plan(idx, nq, nprobe, k);
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
    int32_t *qlist = (int32_t *)(w + pl.off_qlist);
    u64 *partial = (u64 *)(w + pl.off_partial);
    uint32_t *qbound = per_part ? nullptr : (uint32_t *)(w + pl.off_qbound);

    if (ev[0]) LIRA_HIP_TRY(hipEventRecord(ev[0], st));
    // cnt, cursor and head are contiguous at the start of the workspace
    LIRA_HIP_TRY(fill32_async(w, 0u, pl.off_qoff, st));
    if (qbound) LIRA_HIP_TRY(fill32_async(qbound, ~0u, (size_t)nq * 4, st));
    const int64_t npairs = nq * nprobe;
    const int nl = (int)idx->n_lists;
    // Two groups when the pruning bound is on and partitions get >= 32 queries:
    // every query's first probe slot (its nearest partition, where most of its
    // top-k lives) is queued ahead of the other slots, so those start with a
    // tight published bound (measured: they then admit almost no survivors).
    // One launch, so there is no tail between the groups.  With m = ceil(32 *
    // n_lists / nq) > 1 first-slot blocks would be part-filled; measured slower
    // there (GIST1M, BIGANN), so one group.
    const int prune_env = idx->opt.prune;
    const int two_group_env = idx->opt.two_phase;
    const int64_t m1 = (kQT * (int64_t)nl + nq - 1) / nq;
    const bool l2_prune = idx->metric == LIRA_METRIC_L2 && prune_env && !(flags & LIRA_SCAN_NO_PRUNE);
    const int groups = qbound && two_group_env && (m1 == 1 || l2_prune || two_group_env == 2) && nprobe >= 2
                           ? 2 : 1;
    const int split = 1;
    const int nv = groups * nl;
    const unsigned pg = (unsigned)((npairs + kPairsPerBlock - 1) / kPairsPerBlock);
    const size_t hc = nv <= kHistMax ? (size_t)nv * 4 : 0;
    const size_t hf = nv <= kHistMax / 2 ? (size_t)nv * 8 : 0;
    hipLaunchKernelGGL(k_count, dim3(pg), dim3(256), hc, st, probe, npairs, nl, (int)nprobe, split, groups,
                       cnt, idx->err);
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, st, cnt, idx->tile_off, nl, nv, pl.bpc, pl.bpc, kQT, qoff,
                       item_off, nch, head, (int32_t *)nullptr, (int4 *)nullptr, pl.bpc, 1, 4, 0);
    hipLaunchKernelGGL(k_fill, dim3(pg), dim3(256), hf, st, probe, npairs, nl, (int)nprobe, split, groups,
                       qoff, cursor, qlist);
    LIRA_HIP_TRY(hipGetLastError());

    ScanArgs a;
    a.Q = q;
    a.X = idx->X;
    a.ids = idx->ids;
    a.tile_off = idx->tile_off;
    a.cnt = cnt;
    a.qoff = qoff;
    a.qlist = qlist;
    a.item_off = item_off;
    a.nch = nch;
    a.head = head;
    a.partial = partial;
    a.qbound = qbound;
    a.d = idx->d;
    a.dpad = idx->dpad;
    a.n_lists = nl;
    a.n_virt = nv;
    a.nprobe = (int)nprobe;
    a.k = (int)k;
    a.bpc = pl.bpc;
    a.nch_max = pl.nch_max;
    a.prune = prune_env && !(flags & LIRA_SCAN_NO_PRUNE);
    a.stats = idx->stats_on ? (unsigned long long *)idx->stats : nullptr;
    a.pivot = idx->pivot;
    a.tstat = idx->tstat;
    if (ev[1]) LIRA_HIP_TRY(hipEventRecord(ev[1], st));
    const bool fma = (flags & LIRA_SCAN_FMA) != 0;
    hipError_t e;
    if (idx->metric == LIRA_METRIC_L2)
        e = fma ? launch_scan_rl<LIRA_METRIC_L2, true>(RL, a, pl, st)
                : launch_scan_rl<LIRA_METRIC_L2, false>(RL, a, pl, st);
    else
        e = fma ? launch_scan_rl<LIRA_METRIC_IP, true>(RL, a, pl, st)
                : launch_scan_rl<LIRA_METRIC_IP, false>(RL, a, pl, st);
    if (e != hipSuccess) return fail(LIRA_EHIP, std::string("k_scan launch: ") + hipGetErrorString(e));
    if (ev[2]) LIRA_HIP_TRY(hipEventRecord(ev[2], st));

    MergeArgs m;
    m.partial = partial;
    m.probe = probe;
    m.nch = nch;
    m.list_size = idx->list_size;
    m.D = out_D;
    m.I = out_I;
    m.ncand = out_ncand;
    m.nq = nq;
    m.n_lists = nl;
    m.nprobe = (int)nprobe;
    m.k = (int)k;
    m.nch_max = pl.nch_max;
    m.metric = idx->metric;
    m.dedup = dedup ? 1 : 0;
    m.per_partition = per_part ? 1 : 0;
    switch (Rm) {
        case 1: launch_merge<1>(m, st); break;
        case 2: launch_merge<2>(m, st); break;
        case 4: launch_merge<4>(m, st); break;
        default: launch_merge<8>(m, st); break;
    }
    LIRA_HIP_TRY(hipGetLastError());
    if (ev[3]) LIRA_HIP_TRY(hipEventRecord(ev[3], st));
    return LIRA_OK;
}

std::string screen_describe(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags);

std::string scan_describe(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags) {
    if (use_screen(idx, k, flags)) return screen_describe(idx, nq, nprobe, k, flags);
    if (!idx->X) return "unsupported (needs the fp32 tiles)";
    ScanPlan pl = make_plan(idx, nq, nprobe, k);
    return std::string("k_scan exact VALU") + ((flags & LIRA_SCAN_FMA) ? " FMA" : "") + " RL=" +
           std::to_string(scan_rl(k)) + " grid=" + std::to_string(pl.grid) + " smem=" + std::to_string(pl.smem);
}

int scan_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe, int64_t nprobe,
              int64_t k, unsigned flags, float *out_D, int64_t *out_I, int64_t *out_ncand,
              void *ws, size_t ws_bytes, hipStream_t st) {
    const bool dedup = (flags & LIRA_SCAN_DEDUP) != 0;
    const bool per_part = (flags & LIRA_SCAN_PER_PARTITION) != 0;
    int64_t kpm = std::max<int64_t>(64, per_part ? k : (dedup ? k * std::max(1, idx->max_replicas) : k));
    int Rm = merge_r(kpm);
    if (Rm < 0)
        return fail(LIRA_EUNSUPPORTED,
                    "k * max_replicas = " + std::to_string(k * idx->max_replicas) +
                        " exceeds the 512-key merge list");
    if (nq == 0) return LIRA_OK;
    if (nq * nprobe > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "nq * nprobe_max must be < 2^31");
    const bool scr = use_screen(idx, k, flags);
    if (!scr && !idx->X)
        return fail(LIRA_EUNSUPPORTED, (flags & (LIRA_SCAN_FMA | LIRA_SCAN_EXACT))
                                           ? "LIRA_SCAN_EXACT / LIRA_SCAN_FMA need the fp32 tiles (LIRA_OPT_KEEP_TILES)"
                                           : "k = " + std::to_string(k) +
                                                 " needs the fp32 tiles (LIRA_OPT_KEEP_TILES) or k <= 120");
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t ev_slot = 0;
    {
        std::lock_guard<std::mutex> lock(idx->mu);
        if (idx->profiling) {
            while (idx->ev_pool.size() < idx->ev_used + 4) {
                hipEvent_t e;
                LIRA_HIP_TRY(hipEventCreate(&e));
                idx->ev_pool.push_back(e);
            }
            ev_slot = idx->ev_used;
            for (int i = 0; i < 4; ++i) ev[i] = idx->ev_pool[ev_slot + i];
            idx->ev_used += 4;
        }
        if (idx->stats_on) idx->stats_paths |= scr ? 2 : 1;
    }
    int rc = scr ? screen_topk(idx, q, nq, probe, nprobe, k, flags, Rm, out_D, out_I, out_ncand, ws, ws_bytes, st, ev)
                 : exact_topk(idx, q, nq, probe, nprobe, k, flags, Rm, out_D, out_I, out_ncand, ws, ws_bytes, st, ev);
    if (rc == LIRA_OK && !ws) rc = cached_workspace_enqueued(idx, st);
    if (rc != LIRA_OK && ev[0]) {
        // this call's events were not all recorded: drop its slots if they are the
        // pool's last (another stream's call may have taken later ones meanwhile),
        // else record all four now, so the read sees a valid zero-length call
        std::lock_guard<std::mutex> lock(idx->mu);
        if (idx->ev_used == ev_slot + 4)
            idx->ev_used = ev_slot;
        else
            for (int i = 0; i < 4; ++i) hipEventRecord(ev[i], st);
    }
    return rc;
}

// Plan kernels for another scan kernel (lira_screen.hip): `groups` groups of
// virtual partitions (2: every query's first probe slot ahead of the rest),
// `qr` queries per item, query-block offsets in qblk_off; group 0's buckets
// are cut into chunks of bpc_near blocks, the rest into chunks of bpc.
// cnt, cursor and head must be zeroed by the caller.
hipError_t launch_plan(const lira_index *idx, const int32_t *probe, int64_t npairs, int nprobe, int bpc,
                       int bpc_near, int qr, int groups, int32_t *cnt, int32_t *cursor, int32_t *qoff, int32_t *item_off,
                       int32_t *nch, int32_t *head, int32_t *qlist, int32_t *qblk_off, int4 *itab,
                       hipStream_t st, int bpc_near_min, int workers, int near_div, int near0,
                       const int32_t *cnt8) {
    const int nl = (int)idx->n_lists, nv = groups * nl;
    const unsigned pg = (unsigned)((npairs + kPairsPerBlock - 1) / kPairsPerBlock);
    const size_t hc = nv <= kHistMax ? (size_t)nv * 4 : 0;
    const size_t hf = nv <= kHistMax / 2 ? (size_t)nv * 8 : 0;
    // (cnt8: the seed already counted every live pair, per XCD -- k_seed_p; the fused
    // plan sums the 8 replicas into cnt)
    const bool counted = cnt8 && nv <= kFuseMax && qblk_off;
    if (!counted) hipLaunchKernelGGL(k_count, dim3(pg), dim3(256), hc, st, probe, npairs, nl, nprobe, 1, groups, cnt, idx->err);
    if (nv <= kFuseMax && qblk_off) {
        hipLaunchKernelGGL(k_plan_fill, dim3(pg + 1), dim3(1024), 0, st, probe, npairs, nl, nprobe, groups, cnt,
                           idx->tile_off, bpc, bpc_near, qr, qoff, item_off, nch, head, qblk_off, itab, cursor, qlist,
                           bpc_near_min, workers, near_div, near0, counted ? cnt8 : nullptr);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, st, cnt, idx->tile_off, nl, nv, bpc, bpc_near, qr, qoff,
                       item_off, nch, head, qblk_off, itab, bpc_near_min, workers, near_div, near0);
    hipLaunchKernelGGL(k_fill, dim3(pg), dim3(256), hf, st, probe, npairs, nl, nprobe, 1, groups, qoff, cursor,
                       qlist);
    return hipGetLastError();
}

}  // namespace lira
