// k-way merge of per-shard top-k lists: the exchange step of the partition-
// sharded search ("shard by partition ... all-gather 8 x (nq, k)
// and k-way merge").  Each rank scans only the lists it owns for every query;
// its (nq, k) result is the exact top-k over its candidates, so the k smallest
// (score, id) keys of the union of the P ranks' lists are the single-GPU
// result: search.cpp:495-514's top-k (nth_element + sort on (score, id)) over
// the same candidates, with the module's replica dedup (Appendix A) applied
// across shards the same way as within one (a row sitting in buckets of two
// shards yields the same key twice, adjacent in merge order).
//
// One wave per query, lane p = shard p's head: every output slot is a wave-wide
// min over the heads (6 u64 shuffle steps), and the winning lane advances.
#include <string>

#include "lira_device.hpp"
#include "lira_internal.hpp"

namespace lira {

// the scan's output convention -> its ordering key (emit_key's inverse):
// L2 ascending D, IP descending D; ties -> smaller id; I = -1 pads
__device__ __forceinline__ u64 out_key(float D, int64_t I, int metric) {
    if (I < 0) return kEmptyKey;
    return make_key(metric == LIRA_METRIC_IP ? -D : D, (int32_t)I);
}

__global__ __launch_bounds__(256) void k_merge_shards(const float *D, const int64_t *I, int nparts, int64_t nq,
                                                      int k, int metric, int dedup, float *outD,
                                                      int64_t *outI) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;  // (wave-uniform)
    const int64_t stride = nq * (int64_t)k;  // one shard's (nq, k) block
    const float *dp = D + (int64_t)lane * stride + q * k;
    const int64_t *ip = I + (int64_t)lane * stride + q * k;
    int pos = 0;
    u64 head = lane < nparts ? out_key(dp[0], ip[0], metric) : kEmptyKey;
    u64 last = kEmptyKey;
    int out = 0;
    while (out < k) {
        u64 m = head;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) m = kmin(m, shfl_xor64(m, s));
        if (m == kEmptyKey) break;  // every shard exhausted
        // the lowest lane holding the minimum advances (equal keys: one per round)
        const u64 own = __ballot(head == m);
        const int win = __builtin_ctzll(own);
        if (!(dedup && m == last)) {
            if (lane == 0) emit_key(m, metric, outD + q * k + out, outI + q * k + out);
            ++out;
            last = m;
        }
        if (lane == win) {
            ++pos;
            head = pos < k ? out_key(dp[pos], ip[pos], metric) : kEmptyKey;
        }
    }
    for (int e = out + lane; e < k; e += 64) emit_key(kEmptyKey, metric, outD + q * k + e, outI + q * k + e);
}

}  // namespace lira

using namespace lira;

extern "C" {

int lira_merge_shards(const float *D, const int64_t *I, int64_t nparts, int64_t nq, int64_t k, int metric,
                      int dedup, float *out_D, int64_t *out_I, void *stream) {
    if (nparts <= 0 || nparts > 64) return fail(LIRA_EINVAL, "nparts must be 1..64");
    if (nq < 0 || k <= 0 || k > 4096) return fail(LIRA_EINVAL, "bad shape");
    if (metric != LIRA_METRIC_L2 && metric != LIRA_METRIC_IP) return fail(LIRA_EINVAL, "unknown metric");
    if (nq == 0) return LIRA_OK;
    if (!D || !I || !out_D || !out_I) return fail(LIRA_EINVAL, "NULL buffer");
    if ((nq + 3) / 4 > INT32_MAX) return fail(LIRA_EUNSUPPORTED, "too many queries for one launch");
    hipLaunchKernelGGL(k_merge_shards, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, (hipStream_t)stream, D, I,
                       (int)nparts, nq, (int)k, metric, dedup ? 1 : 0, out_D, out_I);
    LIRA_HIP_TRY(hipGetLastError());
    return LIRA_OK;
}

}  // extern "C"
