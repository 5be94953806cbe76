// lira_internal.hpp -- host-side state shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "lira_hip.h"

namespace lira {

// thread-local message behind lira_last_error()
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
// true only when lira_screen.hip is compiled with -DLIRA_DEBUG (or -DLIRA_PHASE_CLOCKS):
// then LIRA_OPT_DEBUG's result-invalidating timing switches are accepted
bool debug_build();

#define LIRA_HIP_TRY(expr)                                                                     \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return ::lira::fail(LIRA_EHIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
    } while (0)

// HBM layout of the partitioned base vectors.
//   X    : [n_tiles][dpad][64] fp32   -- 64 candidates per tile, d-major, so a
//          wave reading dims j..j+3 of a tile reads 1 KiB contiguous; dims in
//          [d, dpad) are zero (dpad = d rounded up to kDimChunk).
//   ids  : [n_tiles*64] int32 global row ids, -1 for the padding slots.
//   tile_off[b]..tile_off[b+1]: the tiles of bucket b; list_size[b]: its rows.
static constexpr int kTile = 64;
static constexpr int kDimChunk = 32;

// lira_index_set_option values (include/lira_hip.h LIRA_OPT_*)
struct lira_opts {
    int keep_tiles = 1;
    int screen = 1;
    int split = 1;
    int qr = 0;
    int two_phase = 1;
    int prune = 1;
    int seed = 1;
    int share = 1;
    int rounds = 0;
    int near_rounds = 0;  // 0: auto (the plan sizes group 0 from the seed's work estimate, between 2 and 6 rounds)
    int mfma = 1;
    int debug = 0;
    int probes_hint = 0;
    int xhi = -1;
    int order = 1;
    int rscreen = 1;
    int near_first = -1;  // LIRA_OPT_NEAR_FIRST (-1: the default, 4 blocks)
    int rescan = -1;      // LIRA_OPT_RESCAN (-1: auto)
    int spill = -1;       // LIRA_OPT_SPILL (-1: 256 records per query)
    int seed_tiles = 0;   // LIRA_OPT_SEED_TILES (0: auto)
    int chunk = 0;        // LIRA_OPT_CHUNK (0: auto)
    int ip_centre = 1;    // LIRA_OPT_IP_CENTRE (build time): IP lists centred on their pivots like L2's
};

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// `mask` is the kernel's own latch, one bit per device ordinal.
hipError_t set_smem_attr_once(std::atomic<uint64_t> &mask, const void *fn, int bytes);

struct lira_index_impl {
    lira_opts opt;
    int device = 0;
    int64_t d = 0, dpad = 0;
    int metric = LIRA_METRIC_L2;
    int64_t n_lists = 0, ntotal = 0, n_tiles = 0, max_list = 0, max_list_tiles = 0;
    int32_t max_replicas = 1;
    std::vector<int64_t> h_list_size, h_tile_off;
    float *X = nullptr;
    int32_t *ids = nullptr;
    int32_t *tile_off = nullptr;   // n_lists+1 (int32: < 2^31 tiles)
    int32_t *list_size = nullptr;  // n_lists
    // For the scan's block skips (L2: triangle inequality; IP: Cauchy-Schwarz on
    // the centred copy): per-list pivot (mean of its rows, fp32, n_lists x d) and
    // per-tile radius bounds (lo, hi) with lo <= ||x - pivot|| <= hi for every
    // real row of the tile.  L2 always; IP where the index is centred (ipc).
    float *pivot = nullptr;
    float2 *tstat = nullptr;
    // per list: (min, max) of its tiles' radius ranges (the scan's pair filter)
    float2 *lstat = nullptr;
    float2 *lsamp = nullptr;  // [n_lists][16] radius ranges of 16 evenly spaced tiles (k_list_stats): the seed's work estimate
    // For the screened scan (lira_screen.hip): per storage row xadj = ||x||^2 / 2
    // (L2, the fp32 rounding of the double sum, halved) or 0 (IP), +inf for
    // padding rows; per list rmax >= max ||x|| over its rows (rounded up).
    float *xadj = nullptr;
    float *rmax = nullptr;
    // The same for the split-bf16 copy, which holds x - pivot of its list (L2:
    // the screen works on centred vectors, whose norms and hence error bounds
    // are smaller): xadjc = ||fl(x - c)||^2 / 2, rmaxc >= max ||fl(x - c)||.
    // IP centred (ipc): the copy holds fl(x - c) too, xadjc = 0 (+inf padding)
    // and q.x = q.fl(x - c) + q.c is screened by k_screen_r only (the other
    // screens then take the fp32 tiles); NULL for an uncentred IP index.
    float *xadjc = nullptr;
    float *rmaxc = nullptr;
    bool ipc = false;
    // Row-major copy of the tiles, [n_tiles*64][d] fp32 by storage row: the
    // screened path's exact re-check reads one candidate's d values
    // contiguously (a tile column would cost one cache line per value).
    float *Xr = nullptr;
    // Split-bf16 copy of the tiles for the MFMA screen (lira_abi.hip
    // k_split_tiles; layout at k_screen_m<..., SPLIT>): same bytes as X.
    uint16_t *Xb = nullptr;
    // per tile: max over its rows of ||x - hi(x)|| for the values Xb splits (L2:
    // x - pivot), rounded up -- the hi-only screen's error bound per block
    float *tres = nullptr;
    int32_t *err = nullptr;        // device error word
    // Cached scan workspaces (workspace == NULL calls), one per stream: two streams
    // searching one handle concurrently never share a buffer (plan counters, item
    // tables, row lists, bounds).  At most kMaxWsStreams streams hold one at a time;
    // an entry whose last call has completed (its `done` event) and that no captured
    // graph uses is handed to a new stream, else the call returns LIRA_ESTATE.
    struct WsEntry {
        hipStream_t st = nullptr;
        void *p = nullptr;
        size_t bytes = 0;
        bool in_graph = false;       // a stream capture recorded kernels that use p
        hipEvent_t done = nullptr;   // recorded after the last eager call that used p
    };
    static constexpr int kMaxWsStreams = 8;
    std::vector<WsEntry> ws_list;
    std::vector<void *> ws_retired;  // outgrown workspaces a captured graph may still use (freed at destroy)
    // guards the host-side state that concurrent calls on one handle touch:
    // ws_list / ws_retired, the profiling event pool and stats_paths
    std::mutex mu;
    // profiling: 4 events per recorded call (start, after plan, after scan, after merge)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    // scan work counters (lira_index_set_stats): 8 u64 on the device
    bool stats_on = false;
    uint64_t *stats = nullptr;
    int stats_paths = 0;  // scan paths counted since the last read: 1 all-exact, 2 screened
};

int64_t round_up(int64_t x, int64_t m);

// The handle's cached scan workspace of stream `st`, at least `need` bytes.
// Growing it while `st` is being captured is refused (LIRA_EINVAL: the graph would
// bake in an allocation made mid-capture); a workspace that a captured graph uses
// is never freed when a later eager call outgrows it (retired until destroy), so a
// replay after such a call reads valid memory.  LIRA_ESTATE when kMaxWsStreams
// other streams hold workspaces that are still in use.
int cached_workspace(lira_index_impl *idx, size_t need, hipStream_t st, void **out);
// after a call's kernels that use st's cached workspace are enqueued: record its
// `done` event (eager calls only), so the entry can pass to another stream later
int cached_workspace_enqueued(lira_index_impl *idx, hipStream_t st);

}  // namespace lira

struct lira_index : lira::lira_index_impl {};
