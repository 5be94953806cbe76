// lira_rscreen.hpp -- arguments of the wave-streaming screen k_screen_r
// (lira_rscreen.hip), filled by screen_topk (lira_screen.hip).
#pragma once
#include "lira_device.hpp"

namespace lira {

struct RArgs {
    int metric;              // LIRA_METRIC_L2, or LIRA_METRIC_IP on a centred index (lira_index::ipc)
    const char *Xb;          // split-bf16 copy (bytes) of x' = fl(x - c): per tile and 16-dim chunk 4 KiB [g 4][p 64][8 bf16]
    const float *xadj;       // per storage row: L2 fl(||x'||^2)/2, IP 0 (+inf: padding)
    const float *rmax;       // per list: max ||x'|| (centred)
    const float *rmaxx;      // per list: max ||x|| (IP: the exact sum's rounding term)
    const float2 *tstat;     // per tile: lo <= ||x - c|| <= hi (NULL: no triangle / Cauchy-Schwarz skip)
    const float *tres;       // per tile: max ||x' - hi(x')||
    const int32_t *tile_off, *cnt, *qoff, *qlist;
    const int4 *itab;        // item -> (virtual partition, query block, chunk, -)
    int32_t *head;           // plan counters / XCD queue bounds (k_plan)
    const float4 *QN;        // per pair: qn = fl(||q'||^2), ||q'|| (up), pair, fl(||q - c||); IP: qc = fl(q.c), ||q|| (up), pair, qc
    const float *QE;         // per pair: ||q' - hi(q')|| (up)
    const uint16_t *QH;      // per pair: hi(q') as bf16, dpad dims
    u64 *partial;            // [pair][nch_max][32 RL] row lists (k_smerge's input)
    float *pE;               // [pair][nch_max] each list's screening-error bound
    uint32_t *qbound;        // [nq] f2ord(bound on the final k-th exact score)
    int64_t d, dpad;
    int n_lists, n_virt, nprobe, k, bpc, nch_max;
    float gP;                // >= 1 + (d + 4) 2^-24 (bound_P's factor, rounded up)
    float invF;              // >= 1 / (1 - (d + 4) 2^-24) (s_lim's factor, rounded up)
    unsigned long long *stats;
    int32_t *done0;          // per query block: its nearest partition's first chunk is done (NULL: no waits)
    uint4 *spill;            // NULL, or [nq][scap] evicted keys k_smerge may need: (key lo, key hi, E bits, 0)
    unsigned *scnt;          // [nq] records spilled (> scap: overflowed)
    int scap;
};

// k_seed_r: the per-query starting bound from the split copy (hi x hi MFMA screen of
// the first NT tiles of the query's nearest list, bound by errE_r) fused with the
// per-pair records and the partition filter -- the k_screen_r path's seed
struct RSeedArgs {
    int metric;
    const float *Q;
    const int32_t *probe;
    int nprobe, n_lists;
    const int32_t *tile_off;
    const char *Xb;
    const float *xadj, *rmax, *rmaxx;  // centred xadj / rmax, max ||x|| (IP)
    const float2 *tstat;
    const float *tres;
    const float *pivot;
    const float2 *lstat;  // the partition filter (NULL: none)
    int32_t *probe_live;
    float4 *QN;
    float *QE, *pqn;
    uint16_t *QH;
    const int32_t *list_size;  // (non-null) the work estimate, as k_seed_t
    const float2 *lsamp;
    unsigned int *work;
    uint32_t *qbound;
    int64_t d, dpad, nq;
    int k;
    int records;  // 1: the records of slots 1.. too; 0: slot 0 only (k_pairs takes the rest)
};
// nt: tiles of 64 rows (1, 2 or 4; 64 nt >= k)
hipError_t launch_seed_r(const RSeedArgs &a, int nt, hipStream_t st);

// the shapes k_screen_r implements: L2 or IP on the centred split copy, hi x hi,
// k <= 120 (row lists of 32 RL keys, RL = 1 / 2 / 4 for k <= 24 / 56 / 120; 64
// query rows per item at RL 1, else 32), dpad <= 128 (the rows' hi parts in LDS)
bool rscreen_shape_ok(int64_t dpad, int64_t k);
// (RL 4 also as one 8-wave workgroup per CU with 64 rows per item: waves = 8)
int rscreen_smem(int rl, int waves);
int rscreen_qr(int rl, int waves);
hipError_t launch_rscreen(const RArgs &a, int rl, int waves, int grid, hipStream_t st);

}  // namespace lira
