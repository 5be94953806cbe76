// lira_abi.hip -- the extern "C" boundary of liblira_hip.so (include/lira_hip.h)
// and the partitioned-index object: gathering x_d rows into the HBM tile layout
// (replaces search.cpp:387-403 and faiss index.add per bucket, utils.py:413-420).
#include <algorithm>
#include <new>
#include <cstring>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

hipError_t set_smem_attr_once(std::atomic<uint64_t> &mask, const void *fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = dev < 64 ? 1ull << dev : 0;
    if (bit && (mask.load(std::memory_order_acquire) & bit)) return hipSuccess;
    // idempotent: two threads racing here both set the same attribute
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess && bit) mask.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// scan entry points (lira_scan.hip)
int scan_workspace_size(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags, size_t *bytes);
std::string scan_describe(const lira_index *idx, int64_t nq, int64_t nprobe, int64_t k, unsigned flags);
int scan_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe, int64_t nprobe,
              int64_t k, unsigned flags, float *out_D, int64_t *out_I, int64_t *out_ncand,
              void *ws, size_t ws_bytes, hipStream_t st);

// Build order (row-major first, so the fp32 tile copy is optional):
//   Xr  [n_tiles*64][d] fp32 by storage row = x[list_ids] (k_row_gather); the
//       screened path's exact re-check and k_seed read it, and every other
//       copy / statistic below is derived from it;
//   Xb  the split-bf16 screen copy (k_split_rows);
//   X   [n_tiles][dpad][64] fp32 d-major tiles (k_tiles_from_rows), only with
//       LIRA_OPT_KEEP_TILES: read by the all-exact scan and the VALU screen.
// Storage row of a list's r-th row: tile_off[b]*64 + r; rows past the list's
// end (padding) are zero with id -1.

// one workgroup per tile, a wave per row, lanes along the row (coalesced)
__global__ __launch_bounds__(256) void k_row_gather(const float *x, int64_t d, const int32_t *list_ids,
                                                    const int64_t *list_off, const int32_t *tile_off,
                                                    const int32_t *tile_list, int64_t n_tiles, float *Xr,
                                                    int32_t *ids) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const int b = tile_list[t];
        const int64_t n = list_off[b + 1] - list_off[b];
        const int64_t r0 = (t - tile_off[b]) * kTile;
        for (int r = w; r < kTile; r += 4) {
            const bool valid = r0 + r < n;
            const int32_t gid = valid ? list_ids[list_off[b] + r0 + r] : -1;
            const float *src = x + (int64_t)(valid ? gid : 0) * d;
            float *dst = Xr + (t * kTile + r) * d;
            for (int64_t j = lane; j < d; j += 64) dst[j] = valid ? src[j] : 0.0f;
            if (lane == 0) ids[t * kTile + r] = gid;
        }
    }
}

// Pivot of list b = mean of its rows, in double.  Pass 1: per segment of
// kPivSeg rows of one list, per-dim sums (threads along the row: coalesced);
// pass 2 adds a list's segments in order (deterministic).
static constexpr int kPivSeg = 4096;
__global__ __launch_bounds__(256) void k_pivot_partial(const float *Xr, int64_t d, const int32_t *seg_list,
                                                       const int32_t *seg_first, const int32_t *tile_off,
                                                       const int64_t *list_off, double *psum) {
    const int s = blockIdx.x, b = seg_list[s];
    const int64_t j = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
    if (j >= d) return;
    const int64_t n = list_off[b + 1] - list_off[b];
    const int64_t r0 = (int64_t)(s - seg_first[b]) * kPivSeg, r1 = min(n, r0 + kPivSeg);
    const float *base = Xr + (int64_t)tile_off[b] * kTile * d + j;
    double acc = 0.0;
#pragma unroll 8
    for (int64_t r = r0; r < r1; ++r) acc += (double)base[r * d];
    psum[(int64_t)s * d + j] = acc;
}
__global__ __launch_bounds__(256) void k_pivot_final(int64_t d, const int32_t *seg_first, const int64_t *list_off,
                                                     const double *psum, float *pivot) {
    const int b = blockIdx.x;
    const int64_t j = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
    if (j >= d) return;
    double s = 0.0;
    for (int g = seg_first[b]; g < seg_first[b + 1]; ++g) s += psum[(int64_t)g * d + j];
    const int64_t n = list_off[b + 1] - list_off[b];
    pivot[(int64_t)b * d + j] = n > 0 ? (float)(s / (double)n) : 0.0f;
}

// The same pivot read straight from x through the list's ids (list order):
// the radius-ordered build (LIRA_OPT_ORDER) needs it before the row gather.
__global__ __launch_bounds__(256) void k_pivot_partial_ids(const float *x, int64_t d, const int32_t *list_ids,
                                                           const int32_t *seg_list, const int32_t *seg_first,
                                                           const int64_t *list_off, double *psum) {
    const int s = blockIdx.x, b = seg_list[s];
    const int64_t j = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
    if (j >= d) return;
    const int64_t n = list_off[b + 1] - list_off[b];
    const int64_t r0 = (int64_t)(s - seg_first[b]) * kPivSeg, r1 = min(n, r0 + kPivSeg);
    const int32_t *ids = list_ids + list_off[b];
    double acc = 0.0;
#pragma unroll 8
    for (int64_t r = r0; r < r1; ++r) acc += (double)x[(int64_t)ids[r] * d + j];
    psum[(int64_t)s * d + j] = acc;
}

// Block of 64 threads: thread r walks row r (d floats at x + off, off < 0: a
// row of zeros) in dim order, f(j, value).  Every row is read once and
// coalesced: 32-dim slabs go through LDS (thread l loads dim j0 + (l & 31) of
// rows 2i + (l >> 5)), so the per-row sequential sums below keep their order
// (and bits) while HBM sees each byte once -- the lane-per-row walks they
// replace read a tile's rows 4 B at a time, 64 rows apart (k_row_norms read
// 13.3 GB for SIFT1M's 0.51 GB, profiles/r02_sift1m_mixture_pmc_summary.json).
template <class F>
__device__ __forceinline__ void walk_rows64(const float *x, int64_t d, int64_t off, F &&f) {
    __shared__ float slab[64 * 33];
    __shared__ int64_t roff[64];
    const int l = threadIdx.x;
    roff[l] = off;
    __syncthreads();
    for (int64_t j0 = 0; j0 < d; j0 += 32) {
        const int nj = (int)min<int64_t>(32, d - j0), jj = l & 31;
#pragma unroll 8
        for (int i = 0; i < 32; ++i) {
            const int r = 2 * i + (l >> 5);
            const int64_t o = roff[r];
            slab[r * 33 + jj] = o >= 0 && jj < nj ? x[o + j0 + jj] : 0.0f;
        }
        __syncthreads();
        for (int u = 0; u < nj; ++u) f(j0 + u, slab[l * 33 + u]);
        __syncthreads();
    }
}

// Sort key of every list entry for the radius-ordered build: the bits of
// fl(||x - pivot||) (non-negative floats order as their bits), thread r of a
// 64-thread block = entry 64 blockIdx + r (rows gathered through list_ids);
// its list by binary search over the offsets.
__global__ __launch_bounds__(64) void k_entry_radius(const float *x, int64_t d, const int32_t *list_ids,
                                                     const int64_t *list_off, int64_t n_lists, const float *pivot,
                                                     int64_t total, uint32_t *key) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    int64_t lo = 0;
    if (i < total) {
        int64_t hi = n_lists;  // list_off[lo] <= i < list_off[hi]
        while (hi - lo > 1) {
            const int64_t m = (lo + hi) >> 1;
            if (list_off[m] <= i) lo = m; else hi = m;
        }
    }
    const float *pv = pivot + lo * d;
    double s = 0.0;
    walk_rows64(x, d, i < total ? (int64_t)list_ids[i] * d : -1, [&](int64_t j, float v) {
        const double df = (double)v - (double)pv[j];
        s = __builtin_fma(df, df, s);
    });
    if (i < total) key[i] = __float_as_uint((float)__builtin_sqrt(s));
}

// Every per-row statistic of the screen in ONE read of the row-major copy;
// one 64-thread block per tile, thread r = row r (walk_rows64), sums in double
// in dim order:
//   xadj = fl(||x||^2) / 2 (L2; IP 0), +inf for padding, and the list's rmax
//     >= max ||x|| (atomicMax on the bits of a non-negative float);
//   (pivot, tstat) the tile's radius range lo <= ||x - c|| <= hi over its real
//     rows, rounded outward with a 2^-40 margin ((+inf, -inf) without real rows);
//   (pivot, xadjc) xadjc = fl(||fl(x - c)||^2) / 2 (IP: 0) and the list's rmaxc >= max
//     ||fl(x - c)||, fl(x - c) exactly the values k_split_rows splits;
//   (tres) the tile's max over real rows of ||v - hi(v)||, v = fl(x - c) (or x
//     without a pivot), hi(v) the bf16 part k_split_rows stores first.
// sqrt rounded up with a 2^-40 relative margin (the double sums' error is ~d 2^-53).
__global__ __launch_bounds__(64) void k_row_stats(const float *Xr, const int32_t *ids, int64_t d,
                                                  const int32_t *tile_list, int metric, const float *pivot,
                                                  float *xadj, float *rmax, float2 *tstat, float *xadjc, float *rmaxc,
                                                  float *tres) {
    const int lane = threadIdx.x;
    const int64_t t = blockIdx.x;
    const int b = tile_list[t];
    const float *pv = pivot ? pivot + (int64_t)b * d : nullptr;
    double s = 0.0, sr = 0.0, sc = 0.0, sh = 0.0;
    walk_rows64(Xr, d, (t * kTile + lane) * d, [&](int64_t j, float v) {
        const double dv = (double)v;
        s = __builtin_fma(dv, dv, s);
        float w = v;
        if (pv) {
            const float c = pv[j];
            const double df = dv - (double)c;
            sr = __builtin_fma(df, df, sr);
            w = v - c;
            const double dc = (double)w;
            sc = __builtin_fma(dc, dc, sc);
        }
        if (tres) {
            const double r = (double)w - (double)__uint_as_float(bf16_split_part(w, 0) << 16);
            sh = __builtin_fma(r, r, sh);
        }
    });
    const bool real = ids[t * kTile + lane] >= 0;
    const float xn = (float)s;  // round to nearest
    xadj[t * kTile + lane] = !real ? __builtin_inff() : metric == LIRA_METRIC_L2 ? xn * 0.5f : 0.0f;
    float r = real ? __double2float_ru(__builtin_sqrt(s) * (1.0 + 0x1p-40)) : 0.0f;
    float lo = __builtin_inff(), hi = -__builtin_inff(), rc = 0.0f, m = 0.0f;
    if (pv && tstat) {
        const double R = __builtin_sqrt(sr);
        lo = real ? __double2float_rd(R * (1.0 - 0x1p-40)) : __builtin_inff();
        hi = real ? __double2float_ru(R * (1.0 + 0x1p-40)) : -__builtin_inff();
    }
    if (pv && xadjc) {
        xadjc[t * kTile + lane] = !real ? __builtin_inff() : metric == LIRA_METRIC_L2 ? (float)sc * 0.5f : 0.0f;
        rc = real ? __double2float_ru(__builtin_sqrt(sc) * (1.0 + 0x1p-40)) : 0.0f;
    }
    if (tres) m = real ? __double2float_ru(__builtin_sqrt(sh) * (1.0 + 0x1p-40)) : 0.0f;
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) {
        r = fmaxf(r, __shfl_xor(r, k, 64));
        lo = fminf(lo, __shfl_xor(lo, k, 64));
        hi = fmaxf(hi, __shfl_xor(hi, k, 64));
        rc = fmaxf(rc, __shfl_xor(rc, k, 64));
        m = fmaxf(m, __shfl_xor(m, k, 64));
    }
    if (lane == 0) {
        if (r > 0.0f) atomicMax((unsigned int *)&rmax[b], __float_as_uint(r));
        if (pv && tstat) tstat[t] = make_float2(lo, hi);
        if (pv && xadjc && rc > 0.0f) atomicMax((unsigned int *)&rmaxc[b], __float_as_uint(rc));
        if (tres) tres[t] = m;
    }
}

// Per list: the (min, max) of its tiles' radius ranges (+inf, -inf for an
// empty list) -- one wave per list.
__global__ __launch_bounds__(64) void k_list_stats(const float2 *tstat, const int32_t *tile_off, float2 *lstat,
                                                   float2 *lsamp) {
    const int b = blockIdx.x, lane = threadIdx.x;
    if (lsamp && lane < 16) {  // tile (lane * tiles / 16)'s range ((+inf, -inf) for an empty list)
        const int t0 = tile_off[b], nt = tile_off[b + 1] - t0;
        lsamp[b * 16 + lane] = nt > 0 ? tstat[t0 + (int)(((int64_t)lane * nt) / 16)]
                                      : make_float2(__builtin_inff(), -__builtin_inff());
    }
    float lo = __builtin_inff(), hi = -__builtin_inff();
    for (int t = tile_off[b] + lane; t < tile_off[b + 1]; t += 64) {
        const float2 v = tstat[t];
        lo = fminf(lo, v.x);
        hi = fmaxf(hi, v.y);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, m, 64));
        hi = fmaxf(hi, __shfl_xor(hi, m, 64));
    }
    if (lane == 0) lstat[b] = make_float2(lo, hi);
}

// X[tile][j][row] = Xr[tile*64 + row][j]: one workgroup per tile, LDS
// transpose of 64-dim slabs (reads and writes coalesced); dims d..dpad-1 = 0.
__global__ __launch_bounds__(256) void k_tiles_from_rows(const float *Xr, int64_t d, int64_t dpad, float *X) {
    __shared__ float sl[64][65];
    const int64_t t = blockIdx.x;
    for (int64_t j0 = 0; j0 < dpad; j0 += 64) {
        for (int i = threadIdx.x; i < 64 * 64; i += 256) {
            const int r = i >> 6, jj = i & 63;
            sl[jj][r] = j0 + jj < d ? Xr[(t * kTile + r) * d + j0 + jj] : 0.0f;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 64 * 64; i += 256) {
            const int jj = i >> 6, r = i & 63;
            if (j0 + jj < dpad) X[(t * dpad + j0 + jj) * kTile + r] = sl[jj][r];
        }
        __syncthreads();
    }
}

// Xb: the split-bf16 copy for the MFMA screen (lira_screen.hip
// k_screen_m<..., SPLIT>).  Per tile and 16-dim chunk c, 4 KiB = [g 4][p 64]
// [8 bf16], g = 2 hl + h: the hi (hl = 0) or lo (hl = 1) round-to-nearest
// bf16 part of dims 16c + 8h .. +7 of candidate row 4 (p & 15) + (p >> 4) (the
// permutation makes a 16-lane group's B-fragment reads consecutive).  One
// workgroup per (tile, chunk), one 16-B unit per thread.
// With pivot (L2): the parts of fl(x - c), c = the row's list pivot.
__global__ __launch_bounds__(256) void k_split_rows(const float *Xr, int64_t d, int64_t n_tiles, int64_t dpad,
                                                   const float *pivot, const int32_t *tile_list, uint4 *Xb) {
    const int64_t nch = dpad / 16, total = n_tiles * nch;
    const int u = threadIdx.x, g = u >> 6, p = u & 63, r = 4 * (p & 15) + (p >> 4), h = g & 1, hl = g >> 1;
    for (int64_t tc = blockIdx.x; tc < total; tc += gridDim.x) {
        const int64_t t = tc / nch, c = tc % nch;
        const float *src = Xr + (t * kTile + r) * d;
        const float *pv = pivot ? pivot + (int64_t)tile_list[t] * d : nullptr;
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            uint32_t part[2];
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const int64_t j = 16 * c + 8 * h + 2 * e + f;
                part[f] = bf16_split_part(j < d ? (pv ? src[j] - pv[j] : src[j]) : 0.0f, hl);
            }
            w[e] = part[0] | (part[1] << 16);
        }
        Xb[tc * 256 + u] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__global__ void k_check_ids(const int32_t *ids, int64_t n, int64_t n_rows, int32_t *bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        if (ids[i] < 0 || ids[i] >= n_rows) atomicOr(bad, 1);
}

static void free_storage(lira_index *idx) {
    if (idx->X) hipFree(idx->X);
    if (idx->ids) hipFree(idx->ids);
    if (idx->tile_off) hipFree(idx->tile_off);
    if (idx->list_size) hipFree(idx->list_size);
    if (idx->Xr) hipFree(idx->Xr);
    idx->Xr = nullptr;
    if (idx->Xb) hipFree(idx->Xb);
    idx->Xb = nullptr;
    if (idx->tres) hipFree(idx->tres);
    idx->tres = nullptr;
    if (idx->xadj) hipFree(idx->xadj);
    if (idx->rmax) hipFree(idx->rmax);
    if (idx->xadjc) hipFree(idx->xadjc);
    if (idx->rmaxc) hipFree(idx->rmaxc);
    idx->xadj = nullptr;
    idx->rmax = nullptr;
    idx->xadjc = nullptr;
    idx->rmaxc = nullptr;
    if (idx->pivot) hipFree(idx->pivot);
    if (idx->tstat) hipFree(idx->tstat);
    if (idx->lstat) hipFree(idx->lstat);
    if (idx->lsamp) hipFree(idx->lsamp);
    idx->lsamp = nullptr;
    idx->pivot = nullptr;
    idx->tstat = nullptr;
    idx->lstat = nullptr;
    idx->X = nullptr;
    idx->ids = nullptr;
    idx->tile_off = nullptr;
    idx->list_size = nullptr;
    idx->n_lists = idx->ntotal = idx->n_tiles = idx->max_list = idx->max_list_tiles = 0;
    idx->ipc = false;  // (the centred IP layout went with xadjc / pivot / Xb)
    idx->h_list_size.clear();
    idx->h_tile_off.clear();
}

int cached_workspace(lira_index_impl *idx, size_t need, hipStream_t st, void **out) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    LIRA_HIP_TRY(hipStreamIsCapturing(st, &cs));
    const bool capturing = cs == hipStreamCaptureStatusActive;
    std::lock_guard<std::mutex> lock(idx->mu);
    lira_index_impl::WsEntry *e = nullptr;
    for (auto &x : idx->ws_list)
        if (x.st == st) e = &x;
    if (capturing && (!e || e->bytes < need)) {
        // a capture on a stream of its own (torch.cuda.graph's side stream) after eager
        // calls on another: the graph takes the largest buffer an eager call sized (it
        // cannot allocate mid-capture); its replays then share that buffer with the eager
        // stream's calls -- replay it on that stream, or pass a workspace
        lira_index_impl::WsEntry *b = nullptr;
        for (auto &x : idx->ws_list)
            if (x.bytes >= need && (!b || x.bytes > b->bytes)) b = &x;
        if (b) {
            b->in_graph = true;
            *out = b->p;
            return LIRA_OK;
        }
    }
    if (!e) {
        if ((int)idx->ws_list.size() < lira_index_impl::kMaxWsStreams) {
            idx->ws_list.emplace_back();
            e = &idx->ws_list.back();
        } else {  // hand over an idle entry: its last call completed, no graph uses it
            for (auto &x : idx->ws_list) {
                if (x.in_graph) continue;
                const hipError_t q = x.done ? hipEventQuery(x.done) : hipSuccess;
                if (q == hipSuccess) {
                    e = &x;
                    break;
                }
                if (q != hipErrorNotReady) return fail(LIRA_EHIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
            }
            if (!e)
                return fail(LIRA_ESTATE, "the cached scan workspace is in use on " +
                                             std::to_string(lira_index_impl::kMaxWsStreams) +
                                             " other streams: pass a workspace (lira_scan_workspace_size)");
        }
        e->st = st;
    }
    if (e->bytes < need) {
        if (capturing)
            return fail(LIRA_EINVAL, "the cached scan workspace must grow to " + std::to_string(need) +
                                         " bytes while the stream is being captured: make the same call once "
                                         "before the capture, or pass a workspace");
        if (e->p) {
            if (e->in_graph)
                idx->ws_retired.push_back(e->p);
            else
                hipFree(e->p);
        }
        e->p = nullptr;
        e->bytes = 0;
        e->in_graph = false;
        LIRA_HIP_TRY(hipMalloc(&e->p, need));
        e->bytes = need;
    }
    if (capturing) e->in_graph = true;
    *out = e->p;
    return LIRA_OK;
}

int cached_workspace_enqueued(lira_index_impl *idx, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    LIRA_HIP_TRY(hipStreamIsCapturing(st, &cs));
    if (cs == hipStreamCaptureStatusActive) return LIRA_OK;  // (a graph's entry is never handed over)
    std::lock_guard<std::mutex> lock(idx->mu);
    for (auto &x : idx->ws_list) {
        if (x.st != st) continue;
        if (!x.done) LIRA_HIP_TRY(hipEventCreateWithFlags(&x.done, hipEventDisableTiming));
        LIRA_HIP_TRY(hipEventRecord(x.done, st));
    }
    return LIRA_OK;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
};

}  // namespace lira

using namespace lira;

extern "C" {

int lira_abi_version(void) { return LIRA_ABI_VERSION; }

const char *lira_last_error(void) { return g_last_error.c_str(); }

int lira_device_cu_count(int device, int *out) {
    if (!out) return fail(LIRA_EINVAL, "out is NULL");
    int v = 0;
    LIRA_HIP_TRY(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device));
    *out = v;
    return LIRA_OK;
}

int lira_index_create(int device, int64_t d, int metric, lira_index **out) {
    if (!out) return fail(LIRA_EINVAL, "out is NULL");
    *out = nullptr;
    if (d <= 0) return fail(LIRA_EINVAL, "d must be > 0");
    if (metric != LIRA_METRIC_L2 && metric != LIRA_METRIC_IP)
        return fail(LIRA_EINVAL, "metric must be LIRA_METRIC_L2 or LIRA_METRIC_IP");
    int ndev = 0;
    LIRA_HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
        return fail(LIRA_EINVAL, "device " + std::to_string(device) + " not present");
    DeviceGuard g(device);
    lira_index *idx = new (std::nothrow) lira_index();
    if (!idx) return fail(LIRA_ENOMEM, "host allocation failed");
    idx->device = device;
    idx->d = d;
    idx->dpad = round_up(d, kDimChunk);
    idx->metric = metric;
    if (hipMalloc(&idx->err, 16) != hipSuccess || hipMemset(idx->err, 0, 16) != hipSuccess) {
        delete idx;
        return fail(LIRA_ENOMEM, "hipMalloc of the error word failed");
    }
    *out = idx;
    return LIRA_OK;
}

int lira_index_destroy(lira_index *idx) {
    if (!idx) return LIRA_OK;
    DeviceGuard g(idx->device);
    hipDeviceSynchronize();
    free_storage(idx);
    if (idx->err) hipFree(idx->err);
    for (auto &x : idx->ws_list) {
        if (x.p) hipFree(x.p);
        if (x.done) hipEventDestroy(x.done);
    }
    for (void *w : idx->ws_retired) hipFree(w);
    for (hipEvent_t e : idx->ev_pool) hipEventDestroy(e);
    if (idx->stats) hipFree(idx->stats);
    delete idx;
    return LIRA_OK;
}

int lira_index_add_partitions(lira_index *idx, int64_t n_lists, const int64_t *list_offsets,
                              const int32_t *list_ids, const float *x, int64_t n_rows,
                              int32_t max_replicas, void *stream) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    if (n_lists <= 0 || !list_offsets) return fail(LIRA_EINVAL, "n_lists must be > 0 with offsets");
    if (n_lists >= INT32_MAX) return fail(LIRA_EINVAL, "n_lists must be < 2^31");
    if (n_rows < 0) return fail(LIRA_EINVAL, "n_rows < 0");
    DeviceGuard g(idx->device);
    hipStream_t st = (hipStream_t)stream;
    if (list_offsets[0] != 0) return fail(LIRA_EINVAL, "list_offsets[0] must be 0");
    std::vector<int64_t> size(n_lists), toff(n_lists + 1);
    std::vector<int32_t> toff32(n_lists + 1), size32(n_lists), seg_first(n_lists + 1);
    int64_t tiles = 0, mx = 0, mxt = 0, segs = 0;
    for (int64_t b = 0; b < n_lists; ++b) {
        int64_t n = list_offsets[b + 1] - list_offsets[b];
        if (n < 0) return fail(LIRA_EINVAL, "list_offsets must be non-decreasing");
        if (n > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "bucket larger than 2^31 rows");
        size[b] = n;
        size32[b] = (int32_t)n;
        toff[b] = tiles;
        toff32[b] = (int32_t)tiles;
        seg_first[b] = (int32_t)segs;
        segs += (n + kPivSeg - 1) / kPivSeg;
        int64_t nt = (n + kTile - 1) / kTile;
        tiles += nt;
        mx = std::max(mx, n);
        mxt = std::max(mxt, nt);
    }
    toff[n_lists] = tiles;
    seg_first[n_lists] = (int32_t)segs;
    if (tiles >= INT32_MAX / kTile) return fail(LIRA_EUNSUPPORTED, "more than 2^31 storage rows");
    toff32[n_lists] = (int32_t)tiles;
    const int64_t total = list_offsets[n_lists];
    if (total > 0 && (!list_ids || !x)) return fail(LIRA_EINVAL, "list_ids / x is NULL");
    if (n_rows > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "more than 2^31 base rows (int32 gids)");

    free_storage(idx);
    std::vector<int32_t> tile_list(tiles), seg_list(segs);
    for (int64_t b = 0; b < n_lists; ++b) {
        for (int64_t t = toff[b]; t < toff[b + 1]; ++t) tile_list[t] = (int32_t)b;
        for (int32_t s = seg_first[b]; s < seg_first[b + 1]; ++s) seg_list[s] = (int32_t)b;
    }
    const int64_t d = idx->d, dpad = idx->dpad, rows = std::max<int64_t>(tiles, 1) * kTile;
    // the row-major copy first: everything else derives from it (x may be freed afterwards)
    if (hipMalloc(&idx->Xr, (size_t)rows * d * 4) != hipSuccess ||
        hipMalloc(&idx->ids, (size_t)rows * 4) != hipSuccess ||
        hipMalloc(&idx->tile_off, (n_lists + 1) * 4) != hipSuccess ||
        hipMalloc(&idx->list_size, n_lists * 4) != hipSuccess) {
        free_storage(idx);
        return fail(LIRA_ENOMEM, "hipMalloc of " + std::to_string((size_t)rows * d * 4) +
                                     " bytes for the lists failed");
    }
    int64_t *d_loff = nullptr;
    int32_t *d_tlist = nullptr, *d_bad = nullptr, *d_seg = nullptr, *d_segf = nullptr, *d_sorted = nullptr;
    uint32_t *d_key = nullptr, *d_key2 = nullptr;
    void *d_tmp = nullptr;
    double *d_psum = nullptr;
    // pivots, tile radius ranges and the centred split copy: L2 always; IP where
    // LIRA_OPT_IP_CENTRE asks (with the fp32 tiles kept, which the screens other
    // than k_screen_r then read: they have no centred IP form)
    const bool ipc = idx->metric == LIRA_METRIC_IP && idx->opt.ip_centre && idx->opt.keep_tiles && tiles > 0;
    const bool l2 = (idx->metric == LIRA_METRIC_L2 || ipc) && tiles > 0;
    // radius-ordered lists (LIRA_OPT_ORDER): a list's rows stored by ascending
    // ||x - pivot||, so a tile's radius range is narrow and the triangle /
    // Cauchy-Schwarz skip can drop it (results do not depend on the order)
    const bool order = l2 && idx->opt.order && total > 0;
    const unsigned dy = (unsigned)((d + 255) / 256);
    int rc = LIRA_OK;
    do {
        if (hipMalloc(&d_loff, (n_lists + 1) * 8) != hipSuccess ||
            hipMalloc(&d_tlist, (size_t)std::max<int64_t>(tiles, 1) * 4) != hipSuccess ||
            hipMalloc(&d_bad, 4) != hipSuccess) {
            rc = fail(LIRA_ENOMEM, "hipMalloc of build scratch failed");
            break;
        }
        hipError_t e = hipMemcpyAsync(d_loff, list_offsets, (n_lists + 1) * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(d_tlist, tile_list.data(), tiles * 4, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(idx->tile_off, toff32.data(), (n_lists + 1) * 4, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(idx->list_size, size32.data(), n_lists * 4, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0, 4, st);
        if (e != hipSuccess) {
            rc = fail(LIRA_EHIP, std::string("upload failed: ") + hipGetErrorString(e));
            break;
        }
        if (total > 0) {
            hipLaunchKernelGGL(k_check_ids, dim3(1024), dim3(256), 0, st, list_ids, total, n_rows, d_bad);
            int32_t bad = 0;
            e = hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) {
                rc = fail(LIRA_EHIP, std::string("id check failed: ") + hipGetErrorString(e));
                break;
            }
            if (bad) {
                rc = fail(LIRA_ERANGE, "list_ids holds a row id outside [0, n_rows)");
                break;
            }
        }
        if (l2) {  // pivot (mean of a list's rows, double) and tile radius arrays
            if (hipMalloc(&idx->pivot, (size_t)n_lists * d * 4) != hipSuccess ||
                hipMalloc(&idx->tstat, (size_t)tiles * sizeof(float2)) != hipSuccess ||
                hipMalloc(&idx->lstat, (size_t)n_lists * sizeof(float2)) != hipSuccess ||
                hipMalloc(&idx->lsamp, (size_t)n_lists * 16 * sizeof(float2)) != hipSuccess ||
                hipMalloc(&d_seg, (size_t)std::max<int64_t>(segs, 1) * 4) != hipSuccess ||
                hipMalloc(&d_segf, (size_t)(n_lists + 1) * 4) != hipSuccess ||
                hipMalloc(&d_psum, (size_t)std::max<int64_t>(segs, 1) * d * 8) != hipSuccess) {
                rc = fail(LIRA_ENOMEM, "hipMalloc of the pivot / tile radius arrays failed");
                break;
            }
            e = hipMemcpyAsync(d_seg, seg_list.data(), (size_t)segs * 4, hipMemcpyHostToDevice, st);
            if (e == hipSuccess)
                e = hipMemcpyAsync(d_segf, seg_first.data(), (size_t)(n_lists + 1) * 4, hipMemcpyHostToDevice, st);
            if (e != hipSuccess) {
                rc = fail(LIRA_EHIP, std::string("upload failed: ") + hipGetErrorString(e));
                break;
            }
        }
        const int32_t *gather_ids = list_ids;
        if (order) {
            // pivots from x in list order, then a stable segmented radix sort of
            // each list's ids by radius (ties keep list order)
            if (segs > 0)
                hipLaunchKernelGGL(k_pivot_partial_ids, dim3((unsigned)segs, dy), dim3(256), 0, st, x, d, list_ids,
                                   d_seg, d_segf, d_loff, d_psum);
            hipLaunchKernelGGL(k_pivot_final, dim3((unsigned)n_lists, dy), dim3(256), 0, st, d, d_segf, d_loff,
                               d_psum, idx->pivot);
            size_t tb = 0;
            if (hipMalloc(&d_key, (size_t)total * 4) != hipSuccess ||
                hipMalloc(&d_key2, (size_t)total * 4) != hipSuccess ||
                hipMalloc(&d_sorted, (size_t)total * 4) != hipSuccess) {
                rc = fail(LIRA_ENOMEM, "hipMalloc of the radius-order scratch failed (LIRA_OPT_ORDER = 0 skips it)");
                break;
            }
            hipLaunchKernelGGL(k_entry_radius, dim3((unsigned)((total + 63) / 64)), dim3(64), 0, st, x, d, list_ids,
                               d_loff, n_lists, idx->pivot, total, d_key);
            e = hipGetLastError();
            if (e == hipSuccess)
                e = hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, d_key, d_key2, list_ids, d_sorted,
                                                                 (int)total, (int)n_lists, d_loff, d_loff + 1, 0, 32,
                                                                 st);
            if (e == hipSuccess) e = hipMalloc(&d_tmp, std::max<size_t>(tb, 1));
            if (e == hipSuccess)
                e = hipcub::DeviceSegmentedRadixSort::SortPairs(d_tmp, tb, d_key, d_key2, list_ids, d_sorted,
                                                                 (int)total, (int)n_lists, d_loff, d_loff + 1, 0, 32,
                                                                 st);
            if (e != hipSuccess) {
                rc = fail(LIRA_EHIP, std::string("radius order failed: ") + hipGetErrorString(e));
                break;
            }
            gather_ids = d_sorted;
        }
        if (tiles > 0) {
            const int grid = (int)std::min<int64_t>(tiles, 65536);
            hipLaunchKernelGGL(k_row_gather, dim3(grid), dim3(256), 0, st, x, d, gather_ids, d_loff, idx->tile_off,
                               d_tlist, tiles, idx->Xr, idx->ids);
        }
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            rc = fail(LIRA_EHIP, std::string("row gather failed: ") + hipGetErrorString(e));
            break;
        }
        if (tiles == 0) {  // an empty index: the all-exact kernel (one zero tile) answers with pads
            if (hipMalloc(&idx->X, (size_t)dpad * kTile * 4) != hipSuccess ||
                hipMemsetAsync(idx->X, 0, (size_t)dpad * kTile * 4, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                rc = fail(LIRA_ENOMEM, "hipMalloc of the (empty) tile copy failed");
            break;
        }
        if (hipMalloc(&idx->xadj, (size_t)tiles * kTile * 4) != hipSuccess ||
            hipMalloc(&idx->rmax, (size_t)n_lists * 4) != hipSuccess) {
            rc = fail(LIRA_ENOMEM, "hipMalloc of the row-norm arrays failed");
            break;
        }
        e = hipMemsetAsync(idx->rmax, 0, (size_t)n_lists * 4, st);
        if (e == hipSuccess && l2 && !order) {  // (radius order computed them from x already)
            if (segs > 0)
                hipLaunchKernelGGL(k_pivot_partial, dim3((unsigned)segs, dy), dim3(256), 0, st, idx->Xr, d, d_seg,
                                   d_segf, idx->tile_off, d_loff, d_psum);
            hipLaunchKernelGGL(k_pivot_final, dim3((unsigned)n_lists, dy), dim3(256), 0, st, d, d_segf, d_loff,
                               d_psum, idx->pivot);
            e = hipGetLastError();
        }
        // the split-bf16 screen copy: best effort (without it the screen runs on fp32
        // MFMA / VALU); L2: of x - pivot, with its own (centred) norms; its hi-part
        // residual bounds tres also best effort (without them the hi-only screens
        // bound by 2^-8 R)
        if (hipMalloc(&idx->Xb, (size_t)tiles * kTile * dpad * 4) != hipSuccess) {
            (void)hipGetLastError();
            idx->Xb = nullptr;
        }
        if (idx->Xb && idx->pivot) {
            if (hipMalloc(&idx->xadjc, (size_t)tiles * kTile * 4) != hipSuccess ||
                hipMalloc(&idx->rmaxc, (size_t)n_lists * 4) != hipSuccess) {
                rc = fail(LIRA_ENOMEM, "hipMalloc of the centred row-norm arrays failed");
                break;
            }
            if (e == hipSuccess) e = hipMemsetAsync(idx->rmaxc, 0, (size_t)n_lists * 4, st);
        }
        if (idx->Xb && hipMalloc(&idx->tres, (size_t)tiles * 4) != hipSuccess) {
            (void)hipGetLastError();
            idx->tres = nullptr;
        }
        // every per-row statistic in one coalesced pass over Xr
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_row_stats, dim3((unsigned)tiles), dim3(64), 0, st, idx->Xr, idx->ids, d, d_tlist,
                               idx->metric, l2 ? idx->pivot : nullptr, idx->xadj, idx->rmax, l2 ? idx->tstat : nullptr,
                               idx->xadjc, idx->rmaxc, idx->tres);
            e = hipGetLastError();
        }
        if (e == hipSuccess && l2) {
            hipLaunchKernelGGL(k_list_stats, dim3((unsigned)n_lists), dim3(64), 0, st, idx->tstat, idx->tile_off,
                               idx->lstat, idx->lsamp);
            e = hipGetLastError();
        }
        if (e == hipSuccess && idx->Xb) {
            hipLaunchKernelGGL(k_split_rows, dim3((unsigned)std::min<int64_t>(tiles * (dpad / 16), 1 << 20)),
                               dim3(256), 0, st, idx->Xr, d, tiles, dpad, idx->pivot, d_tlist, (uint4 *)idx->Xb);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            rc = fail(LIRA_EHIP, std::string("row statistics / pivots / split copy failed: ") + hipGetErrorString(e));
            break;
        }
        // the fp32 tile copy for the all-exact / VALU kernels (LIRA_OPT_KEEP_TILES)
        if (e == hipSuccess && idx->opt.keep_tiles) {
            if (hipMalloc(&idx->X, (size_t)tiles * dpad * kTile * 4) != hipSuccess) {
                rc = fail(LIRA_ENOMEM, "hipMalloc of the fp32 tile copy failed (LIRA_OPT_KEEP_TILES = 0 drops it)");
                break;
            }
            hipLaunchKernelGGL(k_tiles_from_rows, dim3((unsigned)tiles), dim3(256), 0, st, idx->Xr, d, dpad, idx->X);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            rc = fail(LIRA_EHIP, std::string("screen / tile copies failed: ") + hipGetErrorString(e));
            break;
        }
        if (!idx->X && !idx->Xb) {
            rc = fail(LIRA_ENOMEM, "neither the split-bf16 screen copy nor the fp32 tiles could be allocated");
            break;
        }
    } while (0);
    if (d_loff) hipFree(d_loff);
    if (d_tlist) hipFree(d_tlist);
    if (d_bad) hipFree(d_bad);
    if (d_seg) hipFree(d_seg);
    if (d_segf) hipFree(d_segf);
    if (d_psum) hipFree(d_psum);
    if (d_key) hipFree(d_key);
    if (d_key2) hipFree(d_key2);
    if (d_sorted) hipFree(d_sorted);
    if (d_tmp) hipFree(d_tmp);
    if (rc != LIRA_OK) {
        free_storage(idx);
        return rc;
    }
    idx->n_lists = n_lists;
    idx->ntotal = total;
    idx->n_tiles = tiles;
    idx->max_list = mx;
    idx->max_list_tiles = mxt;
    idx->max_replicas = std::max<int32_t>(1, max_replicas);
    idx->ipc = ipc && idx->xadjc != nullptr;
    idx->h_list_size = size;
    idx->h_tile_off = toff;
    return LIRA_OK;
}

int lira_index_info(const lira_index *idx, int64_t *d, int *metric, int64_t *n_lists,
                    int64_t *ntotal, int64_t *max_list) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    if (d) *d = idx->d;
    if (metric) *metric = idx->metric;
    if (n_lists) *n_lists = idx->n_lists;
    if (ntotal) *ntotal = idx->ntotal;
    if (max_list) *max_list = idx->max_list;
    return LIRA_OK;
}

int lira_index_list_size(const lira_index *idx, int64_t list_no, int64_t *out) {
    if (!idx || !out) return fail(LIRA_EINVAL, "NULL argument");
    if (list_no < 0 || list_no >= idx->n_lists) return fail(LIRA_ERANGE, "list_no out of range");
    *out = idx->h_list_size[list_no];
    return LIRA_OK;
}

int lira_index_memory(const lira_index *idx, int64_t *bytes) {
    if (!idx || !bytes) return fail(LIRA_EINVAL, "NULL argument");
    const int64_t rows = idx->n_tiles * kTile;
    *bytes = rows * 4 + idx->n_lists * 8 +                                   // ids, tile_off + list_size
             (idx->Xr ? rows * idx->d * 4 : 0) +                               // row-major copy
             (idx->Xb ? rows * idx->dpad * 4 : 0) +                            // split-bf16 copy
             (idx->X ? rows * idx->dpad * 4 : 0) +                             // fp32 tiles (optional)
             (idx->xadj ? rows * 4 + idx->n_lists * 4 : 0) +                   // xadj, rmax
             (idx->xadjc ? rows * 4 + idx->n_lists * 4 : 0) +                  // centred xadj, rmax
             (idx->pivot ? idx->n_lists * idx->d * 4 + idx->n_tiles * 8 + idx->n_lists * 8 : 0) +  // pivots, radii
             (idx->tres ? idx->n_tiles * 4 : 0) +                               // tile hi residuals
             (idx->lsamp ? idx->n_lists * 16 * (int64_t)sizeof(float2) : 0);   // sampled tile radius ranges
    return LIRA_OK;
}

int lira_index_set_option(lira_index *idx, int option, int64_t value) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    lira_opts &o = idx->opt;
    const int v = (int)value;
    auto in = [&](int lo, int hi) { return value >= lo && value <= hi; };
    switch (option) {
        case LIRA_OPT_KEEP_TILES: if (!in(0, 1)) break; o.keep_tiles = v; return LIRA_OK;
        case LIRA_OPT_SCREEN: if (!in(0, 1)) break; o.screen = v; return LIRA_OK;
        case LIRA_OPT_SPLIT: if (!in(0, 1)) break; o.split = v; return LIRA_OK;
        case LIRA_OPT_QR: if (value != 0 && value != 32 && value != 64 && value != 128) break; o.qr = v; return LIRA_OK;
        case LIRA_OPT_TWO_PHASE: if (!in(0, 2)) break; o.two_phase = v; return LIRA_OK;
        case LIRA_OPT_PRUNE: if (!in(0, 1)) break; o.prune = v; return LIRA_OK;
        case LIRA_OPT_SEED:
            if (value == 2 || value == 3)  // (k_seed_b, measured slower: removed in round 4)
                return fail(LIRA_EUNSUPPORTED, "LIRA_OPT_SEED 2 / 3 (block-shared seed) was removed");
            if (!in(0, 1)) break;
            o.seed = v;
            return LIRA_OK;
        case LIRA_OPT_SHARE: if (!in(0, 1)) break; o.share = v; return LIRA_OK;
        case LIRA_OPT_ROUNDS: if (!in(0, 1024)) break; o.rounds = v; return LIRA_OK;
        case LIRA_OPT_NEAR_ROUNDS: if (!in(0, 1024)) break; o.near_rounds = v; return LIRA_OK;
        case LIRA_OPT_MFMA: if (!in(0, 2)) break; o.mfma = v; return LIRA_OK;
        case LIRA_OPT_DEBUG:
            if (!in(0, 255)) break;
            if (v && !debug_build())  // a production build never returns invalid results
                return fail(LIRA_EUNSUPPORTED, "LIRA_OPT_DEBUG needs a library built with -DLIRA_DEBUG");
            o.debug = v; return LIRA_OK;
        case LIRA_OPT_PIPELINE:  // (k_screen_s, k_screen_w, k_screen_v: measured slower, removed in round 4)
        case LIRA_OPT_RING:
        case LIRA_OPT_WIDE:
            if (value == 0) return LIRA_OK;
            return fail(LIRA_EUNSUPPORTED, "option " + std::to_string(option) + " selected a screen variant that was removed");
        case LIRA_OPT_PROBES_HINT: if (!in(0, 1 << 20)) break; o.probes_hint = v; return LIRA_OK;
        case LIRA_OPT_XHI: if (!in(-1, 2)) break; o.xhi = v; return LIRA_OK;
        case LIRA_OPT_ORDER: if (!in(0, 1)) break; o.order = v; return LIRA_OK;
        case LIRA_OPT_RSCREEN: if (!in(0, 2)) break; o.rscreen = v; return LIRA_OK;
        case LIRA_OPT_NEAR_FIRST: if (!in(-1, 128)) break; o.near_first = v; return LIRA_OK;
        case LIRA_OPT_RESCAN: if (!in(-1, 1)) break; o.rescan = v; return LIRA_OK;
        case LIRA_OPT_SPILL: if (!in(-1, 1 << 16)) break; o.spill = v; return LIRA_OK;
        case LIRA_OPT_IP_CENTRE: if (!in(0, 1)) break; o.ip_centre = v; return LIRA_OK;
        case LIRA_OPT_CHUNK: if (!in(0, 1 << 20)) break; o.chunk = v; return LIRA_OK;
        case LIRA_OPT_SEED_TILES:
            if (!in(0, 4) || v == 3) break;
            // 4 tiles exist only in the seeds fused with the per-pair records: k_seed_r
            // (k_screen_r's: L2 or centred IP, d <= 128) and k_seed_t (L2, d <= 256, fp32
            // tiles kept); the unfused seed reads 1 or 2.  Once the index has lists the layout
            // as built decides (idx->ipc, idx->X), before that the options that will build it
            if (v == 4) {
                const bool built = idx->Xr != nullptr;
                const bool cip = built ? idx->ipc : (o.ip_centre && o.keep_tiles);
                const bool tiles = built ? idx->X != nullptr : o.keep_tiles != 0;
                if (!(idx->d <= 128 && (idx->metric == LIRA_METRIC_L2 || cip)) &&
                    !(idx->metric == LIRA_METRIC_L2 && idx->d <= 256 && tiles))
                    return fail(LIRA_EUNSUPPORTED, "LIRA_OPT_SEED_TILES 4 needs a fused seed (L2 or centred IP with "
                                                   "d <= 128, or L2 with d <= 256 and the fp32 tiles)");
            }
            o.seed_tiles = v;
            return LIRA_OK;
        default: return fail(LIRA_EINVAL, "unknown option " + std::to_string(option));
    }
    return fail(LIRA_EINVAL, "value " + std::to_string(value) + " out of range for option " + std::to_string(option));
}

int lira_index_get_option(const lira_index *idx, int option, int64_t *value) {
    if (!idx || !value) return fail(LIRA_EINVAL, "NULL argument");
    const lira_opts &o = idx->opt;
    switch (option) {
        case LIRA_OPT_KEEP_TILES: *value = o.keep_tiles; break;
        case LIRA_OPT_SCREEN: *value = o.screen; break;
        case LIRA_OPT_SPLIT: *value = o.split; break;
        case LIRA_OPT_QR: *value = o.qr; break;
        case LIRA_OPT_TWO_PHASE: *value = o.two_phase; break;
        case LIRA_OPT_PRUNE: *value = o.prune; break;
        case LIRA_OPT_SEED: *value = o.seed; break;
        case LIRA_OPT_SHARE: *value = o.share; break;
        case LIRA_OPT_ROUNDS: *value = o.rounds; break;
        case LIRA_OPT_NEAR_ROUNDS: *value = o.near_rounds; break;
        case LIRA_OPT_MFMA: *value = o.mfma; break;
        case LIRA_OPT_DEBUG: *value = o.debug; break;
        case LIRA_OPT_PIPELINE:
        case LIRA_OPT_RING:
        case LIRA_OPT_WIDE: *value = 0; break;
        case LIRA_OPT_PROBES_HINT: *value = o.probes_hint; break;
        case LIRA_OPT_XHI: *value = o.xhi; break;
        case LIRA_OPT_ORDER: *value = o.order; break;
        case LIRA_OPT_RSCREEN: *value = o.rscreen; break;
        case LIRA_OPT_NEAR_FIRST: *value = o.near_first; break;
        case LIRA_OPT_RESCAN: *value = o.rescan; break;
        case LIRA_OPT_SPILL: *value = o.spill; break;
        case LIRA_OPT_SEED_TILES: *value = o.seed_tiles; break;
        case LIRA_OPT_IP_CENTRE: *value = o.ip_centre; break;
        case LIRA_OPT_CHUNK: *value = o.chunk; break;
        default: return fail(LIRA_EINVAL, "unknown option " + std::to_string(option));
    }
    return LIRA_OK;
}

int lira_index_has_tiles(const lira_index *idx, int *out) {
    if (!idx || !out) return fail(LIRA_EINVAL, "NULL argument");
    *out = idx->X != nullptr;
    return LIRA_OK;
}

int lira_scan_workspace_size(const lira_index *idx, int64_t nq, int64_t nprobe_max, int64_t k,
                             unsigned flags, size_t *bytes) {
    if (!idx || !bytes) return fail(LIRA_EINVAL, "NULL argument");
    if (nq < 0 || nprobe_max <= 0 || k <= 0 || k > 256)
        return fail(LIRA_EINVAL, "need nq >= 0, nprobe_max > 0, 1 <= k <= 256");
    return scan_workspace_size(idx, nq, nprobe_max, k, flags, bytes);
}

int lira_scan_describe(const lira_index *idx, int64_t nq, int64_t nprobe_max, int64_t k, unsigned flags,
                       char *out, size_t out_len) {
    if (!idx || !out || out_len == 0) return fail(LIRA_EINVAL, "NULL argument");
    if (idx->n_lists == 0) return fail(LIRA_ESTATE, "index has no lists (add_partitions first)");
    if (nq < 0 || nprobe_max <= 0 || k <= 0 || k > 256) return fail(LIRA_EINVAL, "need nq >= 0, nprobe_max > 0, 1 <= k <= 256");
    const std::string s = scan_describe(idx, nq, nprobe_max, k, flags);
    const size_t n = std::min(out_len - 1, s.size());
    std::memcpy(out, s.data(), n);
    out[n] = 0;
    return LIRA_OK;
}

int lira_scan_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe,
                   int64_t nprobe_max, int64_t k, unsigned flags, float *out_D, int64_t *out_I,
                   int64_t *out_ncand, void *workspace, size_t workspace_bytes, void *stream) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    if (idx->n_lists == 0) return fail(LIRA_ESTATE, "index has no lists (add_partitions first)");
    if (nq < 0 || nprobe_max <= 0) return fail(LIRA_EINVAL, "need nq >= 0 and nprobe_max > 0");
    if (k <= 0 || k > 256) return fail(LIRA_EUNSUPPORTED, "k must be in [1, 256]");
    if (flags & ~(LIRA_SCAN_DEDUP | LIRA_SCAN_PER_PARTITION | LIRA_SCAN_FMA | LIRA_SCAN_NO_PRUNE | LIRA_SCAN_EXACT | LIRA_SCAN_NO_SPLIT)) return fail(LIRA_EINVAL, "unknown flags");
    if (nq > 0 && (!q || !probe || !out_D || !out_I)) return fail(LIRA_EINVAL, "NULL buffer");
    DeviceGuard g(idx->device);
    return scan_topk(idx, q, nq, probe, nprobe_max, k, flags, out_D, out_I, out_ncand, workspace,
                     workspace_bytes, (hipStream_t)stream);
}

int lira_index_set_profiling(lira_index *idx, int enable) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    std::lock_guard<std::mutex> lock(idx->mu);
    idx->profiling = enable != 0;
    idx->ev_used = 0;
    return LIRA_OK;
}

int lira_index_set_stats(lira_index *idx, int enable) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    DeviceGuard g(idx->device);
    if (enable && !idx->stats) LIRA_HIP_TRY(hipMalloc(&idx->stats, 8 * sizeof(uint64_t)));
    if (enable) {
        LIRA_HIP_TRY(hipDeviceSynchronize());
        LIRA_HIP_TRY(hipMemset(idx->stats, 0, 8 * sizeof(uint64_t)));
    }
    idx->stats_on = enable != 0;
    if (enable) idx->stats_paths = 0;
    return LIRA_OK;
}

int lira_index_stats_paths(const lira_index *idx, int *out) {
    if (!idx || !out) return fail(LIRA_EINVAL, "index or out is NULL");
    std::lock_guard<std::mutex> lock(const_cast<lira_index *>(idx)->mu);
    *out = idx->stats_paths;
    return LIRA_OK;
}

int lira_index_stats_read(lira_index *idx, uint64_t *out8) {
    if (!idx || !out8) return fail(LIRA_EINVAL, "index or out is NULL");
    DeviceGuard g(idx->device);
    for (int i = 0; i < 8; ++i) out8[i] = 0;
    if (!idx->stats) return LIRA_OK;
    LIRA_HIP_TRY(hipDeviceSynchronize());
    LIRA_HIP_TRY(hipMemcpy(out8, idx->stats, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    LIRA_HIP_TRY(hipMemset(idx->stats, 0, 8 * sizeof(uint64_t)));
    idx->stats_paths = 0;
    return LIRA_OK;
}

int lira_index_profile_read(lira_index *idx, double *plan_ms, double *scan_ms, double *merge_ms,
                            int64_t *calls) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    DeviceGuard g(idx->device);
    std::lock_guard<std::mutex> lock(idx->mu);
    double sp = 0, ss = 0, sm = 0;
    const size_t n = idx->ev_used / 4;
    for (size_t c = 0; c < n; ++c) {
        hipEvent_t *e = &idx->ev_pool[4 * c];
        // (each call's own last event: calls on several streams complete in any order)
        LIRA_HIP_TRY(hipEventSynchronize(e[3]));
        float a = 0, b = 0, m = 0;
        LIRA_HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]));
        LIRA_HIP_TRY(hipEventElapsedTime(&b, e[1], e[2]));
        LIRA_HIP_TRY(hipEventElapsedTime(&m, e[2], e[3]));
        sp += a;
        ss += b;
        sm += m;
    }
    idx->ev_used = 0;
    if (plan_ms) *plan_ms = sp;
    if (scan_ms) *scan_ms = ss;
    if (merge_ms) *merge_ms = sm;
    if (calls) *calls = (int64_t)n;
    return LIRA_OK;
}

int lira_index_check(lira_index *idx, void *stream) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    DeviceGuard g(idx->device);
    hipStream_t st = (hipStream_t)stream;
    int32_t e = 0;
    LIRA_HIP_TRY(hipMemcpyAsync(&e, idx->err, 4, hipMemcpyDeviceToHost, st));
    LIRA_HIP_TRY(hipStreamSynchronize(st));
    if (e) {
        LIRA_HIP_TRY(hipMemsetAsync(idx->err, 0, 4, st));
        LIRA_HIP_TRY(hipStreamSynchronize(st));
        return fail(LIRA_ERANGE, "a probe id was >= n_lists (slot skipped)");
    }
    return LIRA_OK;
}

}  // extern "C"
