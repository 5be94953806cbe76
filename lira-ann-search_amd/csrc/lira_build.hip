// lira_build.hip -- device-side inverted-list builder.
//
// Replaces search.cpp:366-385: for every row i and slot j of data_2_bkt
// (N, n_mul; -1 = empty), bucket data_2_bkt[i][j] receives row i; each bucket's
// list is sorted ascending and de-duplicated.  On the device:
//   k_flatten   one (bucket, row) pair per valid slot; a bucket repeated in
//               a row's later slot is dropped (that is the de-duplication);
//               per-bucket counts (LDS histogram), max buckets per row
//   radix sort  stable sort of the pairs by bucket (hipCUB onesweep), so each
//               bucket's rows stay ascending -- the std::sort of :383
// The per-bucket offsets come back to the host (n_lists + 1 ints, the one
// synchronisation), then lira_index_add_partitions gathers x into tiles.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <string>
#include <vector>

#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

static constexpr int kFlatHist = 16384;

__global__ __launch_bounds__(256) void k_flatten(const int32_t *d2b, int64_t n, int n_mul, int n_lists,
                                                 uint32_t *keys, int32_t *vals, int32_t *cnt,
                                                 int32_t *max_rep, int32_t *err) {
    extern __shared__ int32_t hist[];
    const bool lds = n_lists <= kFlatHist;
    if (lds) {
        for (int b = threadIdx.x; b < n_lists; b += blockDim.x) hist[b] = 0;
        __syncthreads();
    }
    int local_rep = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t *row = d2b + i * n_mul;
        int rep = 0;
        for (int j = 0; j < n_mul; ++j) {
            const int32_t b = row[j];
            bool valid = b >= 0;
            if (b >= n_lists) {
                atomicOr(err, 1);
                valid = false;
            }
            for (int jj = 0; jj < j && valid; ++jj) valid = row[jj] != b;
            keys[i * n_mul + j] = valid ? (uint32_t)b : (uint32_t)n_lists;  // invalid sorts last
            vals[i * n_mul + j] = (int32_t)i;
            if (valid) {
                atomicAdd(lds ? &hist[b] : &cnt[b], 1);
                ++rep;
            }
        }
        local_rep = max(local_rep, rep);
    }
    if (local_rep) atomicMax(max_rep, local_rep);
    if (lds) {
        __syncthreads();
        for (int b = threadIdx.x; b < n_lists; b += blockDim.x)
            if (hist[b]) atomicAdd(&cnt[b], hist[b]);
    }
}

}  // namespace lira

using namespace lira;

extern "C" int lira_index_build(lira_index *idx, int64_t n_lists, const int32_t *data_2_bkt, int64_t n,
                                int32_t n_mul, const float *x, void *stream) {
    if (!idx) return fail(LIRA_EINVAL, "index is NULL");
    if (n_lists <= 0 || n_lists >= INT32_MAX) return fail(LIRA_EINVAL, "n_lists must be in [1, 2^31)");
    if (n < 0 || n_mul <= 0) return fail(LIRA_EINVAL, "need n >= 0 and n_mul >= 1");
    if (n > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "more than 2^31 base rows (int32 gids)");
    if (n > 0 && (!data_2_bkt || !x)) return fail(LIRA_EINVAL, "NULL buffer");
    const int64_t m = n * n_mul;
    if (m > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "n * n_mul must be < 2^31");
    hipStream_t st = (hipStream_t)stream;
    int prev = -1;
    if (hipGetDevice(&prev) == hipSuccess && prev != idx->device) hipSetDevice(idx->device);

    uint32_t *keys = nullptr, *keys2 = nullptr;
    int32_t *vals = nullptr, *vals2 = nullptr, *cnt = nullptr;
    void *tmp = nullptr;
    int rc = LIRA_OK;
    std::vector<int32_t> hcnt((size_t)n_lists + 2);
    do {
        const size_t sz = (size_t)std::max<int64_t>(m, 1);
        if (hipMalloc(&keys, sz * 4) != hipSuccess || hipMalloc(&keys2, sz * 4) != hipSuccess ||
            hipMalloc(&vals, sz * 4) != hipSuccess || hipMalloc(&vals2, sz * 4) != hipSuccess ||
            hipMalloc(&cnt, (n_lists + 2) * 4) != hipSuccess) {
            rc = fail(LIRA_ENOMEM, "hipMalloc of the build scratch failed");
            break;
        }
        // cnt[0..n_lists) counts, cnt[n_lists] max replicas, cnt[n_lists+1] error word
        if (hipMemsetAsync(cnt, 0, (n_lists + 2) * 4, st) != hipSuccess) {
            rc = fail(LIRA_EHIP, "memset failed");
            break;
        }
        if (n > 0) {
            const int grid = (int)std::min<int64_t>(2048, (n + 255) / 256);
            const size_t sh = n_lists <= kFlatHist ? (size_t)n_lists * 4 : 0;
            hipLaunchKernelGGL(k_flatten, dim3(grid), dim3(256), sh, st, data_2_bkt, n, (int)n_mul,
                               (int)n_lists, keys, vals, cnt, cnt + n_lists, cnt + n_lists + 1);
            int end_bit = 1;
            while (end_bit < 32 && ((uint64_t)1 << end_bit) <= (uint64_t)n_lists) ++end_bit;
            size_t tb = 0;
            hipcub::DoubleBuffer<uint32_t> dk(keys, keys2);
            hipcub::DoubleBuffer<int32_t> dv(vals, vals2);
            hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dv, (int)m, 0, end_bit, st);
            if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tb, 1));
            if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dv, (int)m, 0, end_bit, st);
            if (e != hipSuccess) {
                rc = fail(LIRA_EHIP, std::string("radix sort: ") + hipGetErrorString(e));
                break;
            }
            if (dv.Current() != vals) std::swap(vals, vals2);  // sorted ids now in `vals`
        }
        if (hipMemcpyAsync(hcnt.data(), cnt, (n_lists + 2) * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = fail(LIRA_EHIP, "copy of bucket counts failed");
            break;
        }
        if (hcnt[n_lists + 1]) {
            rc = fail(LIRA_ERANGE, "bucket id out of range.");  // search.cpp:375-377
            break;
        }
        std::vector<int64_t> off((size_t)n_lists + 1, 0);
        for (int64_t b = 0; b < n_lists; ++b) off[b + 1] = off[b] + hcnt[b];
        rc = lira_index_add_partitions(idx, n_lists, off.data(), vals, x, n, std::max(1, hcnt[n_lists]),
                                       stream);
    } while (0);
    hipFree(keys);
    hipFree(keys2);
    hipFree(vals);
    hipFree(vals2);
    hipFree(cnt);
    if (tmp) hipFree(tmp);
    if (prev >= 0 && prev != idx->device) hipSetDevice(prev);
    return rc;
}

extern "C" int lira_index_list_ids(const lira_index *idx, int64_t list_no, int32_t *out, void *stream) {
    if (!idx || !out) return fail(LIRA_EINVAL, "NULL argument");
    if (list_no < 0 || list_no >= idx->n_lists) return fail(LIRA_ERANGE, "list_no out of range");
    const int64_t n = idx->h_list_size[list_no];
    if (n == 0) return LIRA_OK;
    hipStream_t st = (hipStream_t)stream;
    LIRA_HIP_TRY(hipMemcpyAsync(out, idx->ids + idx->h_tile_off[list_no] * kTile, n * 4,
                                hipMemcpyDeviceToHost, st));
    LIRA_HIP_TRY(hipStreamSynchronize(st));
    return LIRA_OK;
}
