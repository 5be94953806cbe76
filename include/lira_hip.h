/*
 * lira_hip.h -- C-ABI of liblira_hip.so, the MI355X (gfx950) implementation of
 * LIRA's query-time hot path: partition ranking, candidate scan and exact
 * top-k over the probed partitions.
 *
 * Every entry point is extern "C", takes plain pointers and sizes (no torch or
 * HIP C++ types) and returns an int status: LIRA_OK (0) or a negative
 * LIRA_E* code; lira_last_error() returns a thread-local message for the last
 * failure.  No C++ exception crosses this boundary.
 *
 * Pointers documented as "device" are HBM pointers (e.g. torch tensors'
 * data_ptr()); "host" pointers are ordinary CPU memory.  `stream` is a
 * hipStream_t passed as void* (NULL = the null stream).  Compute entry points
 * are stream-ordered and asynchronous unless stated otherwise.
 *
 * What each entry point replaces in the reference (qfshen23/LIRA-ANN-search,
 * file:line) is stated above it.  INTEGRATION.md shows the ctypes binding the
 * reference's Python side would use, and lira_amd/_lib.py is that binding.
 */
#ifndef LIRA_HIP_H
#define LIRA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LIRA_ABI_VERSION 1

/* status codes */
#define LIRA_OK 0
#define LIRA_EINVAL (-1)     /* bad argument (shape, k, metric, null pointer) */
#define LIRA_ERANGE (-2)     /* bucket / probe id out of range */
#define LIRA_ENOMEM (-3)     /* device allocation failed */
#define LIRA_EHIP (-4)       /* HIP runtime error (message has the HIP string) */
#define LIRA_ESTATE (-5)     /* call not valid in the handle's current state */
#define LIRA_EUNSUPPORTED (-6) /* shape outside what the kernels implement */

/* metrics: search.cpp:362-364 / LIRA_smallscale.py:62-66 */
#define LIRA_METRIC_L2 0 /* squared L2, ascending  (search.cpp:253-260, faiss IndexFlatL2) */
#define LIRA_METRIC_IP 1 /* inner product, descending (search.cpp:263-269, faiss IndexFlatIP) */

/* lira_scan_topk flags */
#define LIRA_SCAN_DEDUP 1u         /* keep each gid once (search.cpp:496-514 does not: Appendix A) */
#define LIRA_SCAN_PER_PARTITION 2u /* k best of every probed slot on its own (LIRA_smallscale.py:145-174) */
#define LIRA_SCAN_FMA 4u           /* fused multiply-add accumulation: fewer ops, NOT bit-exact (SURVEY 7
                                      "tolerance fallback": 1e-4 relative, ties may order differently) */
#define LIRA_SCAN_NO_PRUNE 8u      /* L2: compute every candidate to the last dim (no early abandon of
                                      pairs already past the k-th score); same results, for A/B */
#define LIRA_SCAN_EXACT 16u        /* use the all-exact scan (every candidate in search.cpp's arithmetic)
                                      instead of the default FMA screen + exact re-check; same results */
#define LIRA_SCAN_NO_SPLIT 32u     /* screen with the fp32 MFMA (v_mfma_f32_16x16x4_f32) instead of the
                                      split-bf16 one (v_mfma_f32_16x16x32_bf16, wider error bound); same
                                      results, for A/B */

/* lira_select_probes modes */
#define LIRA_PROBE_NEAREST 0      /* nprobe smallest values, ties -> smaller bucket (IVF nprobe) */
#define LIRA_PROBE_THRESHOLD_GE 1 /* score >= thr, argmax fallback (search.cpp:447-466) */
#define LIRA_PROBE_THRESHOLD_GT 2 /* score >  thr, no fallback (LIRA_smallscale.py:206) */
#define LIRA_PROBE_BY_SCORE 16    /* or-ed into a THRESHOLD mode: the same set, in descending score order
                                     (ties -> smaller bucket) instead of ascending bucket; truncation at
                                     max_probe keeps the highest scores; max_probe <= 256 */

typedef struct lira_index lira_index; /* opaque; one handle per device */

/* ---------------------------------------------------------------- misc */
int lira_abi_version(void);
const char *lira_last_error(void);
/* number of compute units of `device` (for launch sizing in callers/tests) */
int lira_device_cu_count(int device, int *out);

/* -------------------------------------------------------------- handle */
/*
 * Create an empty partitioned index for d-dimensional fp32 vectors.
 * Replaces faiss.IndexFlatL2(d) / IndexFlatIP(d) construction
 * (utils.py:415-418) and search.cpp's `std::vector<Bucket> buckets`
 * (search.cpp:273-276, 387-388).
 */
int lira_index_create(int device, int64_t d, int metric, lira_index **out);
int lira_index_destroy(lira_index *idx);

/*
 * Load the inverted lists.  Replaces search.cpp:387-403 (per-bucket contiguous
 * copy of x_d rows) and faiss `index.add(x_d[ids])` per bucket
 * (utils.py:413-420).
 *   n_lists           number of buckets B
 *   list_offsets      host, n_lists+1 int64: bucket b owns list_ids[off[b]:off[b+1]]
 *   list_ids          device int32, global row ids (sorted unique per bucket for
 *                     search.cpp parity; any order is accepted)
 *   x                 device fp32 (n_rows, d) row-major base vectors (x_d)
 * The module gathers x[list_ids] into its own HBM layout (64-row, d-major tiles),
 * so x may be freed afterwards.  max_replicas = the largest number of buckets
 * any one row sits in (data_2_bkt's effective n_mul; 1 without redundancy);
 * it sizes the dedup merge.  Synchronous w.r.t. the host on return.
 */
int lira_index_add_partitions(lira_index *idx, int64_t n_lists, const int64_t *list_offsets,
                              const int32_t *list_ids, const float *x, int64_t n_rows,
                              int32_t max_replicas, void *stream);

/*
 * Device-side inverted-list build + load in one call: search.cpp:366-404.
 * data_2_bkt: device int32 (n, n_mul), -1 = empty slot; every valid bucket id
 * of row i receives i, lists are sorted ascending and de-duplicated
 * (search.cpp:371-385), then gathered like lira_index_add_partitions.
 * max_replicas is derived (largest number of distinct buckets of a row).
 * Returns LIRA_ERANGE for a bucket id >= n_lists (search.cpp:375-377).
 * Synchronous w.r.t. the host on return.
 */
int lira_index_build(lira_index *idx, int64_t n_lists, const int32_t *data_2_bkt, int64_t n,
                     int32_t n_mul, const float *x, void *stream);
/* host copy of one bucket's row ids, in STORAGE order: with LIRA_OPT_ORDER=1 (the L2
 * default) rows are stored by ascending distance to the list's pivot, so this is a
 * permutation of the ids passed to add/build (compare as sets; ordering never
 * changes a search result) */
int lira_index_list_ids(const lira_index *idx, int64_t list_no, int32_t *out_host, void *stream);

/* sizes: ntotal = total rows incl. replicas (faiss .ntotal, LIRA_smallscale.py:171) */
int lira_index_info(const lira_index *idx, int64_t *d, int *metric, int64_t *n_lists,
                    int64_t *ntotal, int64_t *max_list);
/* host copy of one bucket's size (search.cpp:476 `sz`) */
int lira_index_list_size(const lira_index *idx, int64_t list_no, int64_t *out);
/* bytes of HBM the index holds */
int lira_index_memory(const lira_index *idx, int64_t *bytes);

/*
 * Per-handle tuning options (no process environment is read by the library).
 * None of them changes a result: every setting returns the same bits (the one
 * exception, LIRA_OPT_DEBUG, is refused unless the library is built with -DLIRA_DEBUG).
 *   LIRA_OPT_KEEP_TILES  1 (default): keep the fp32 d-major tile copy that the
 *                        all-exact scan (LIRA_SCAN_EXACT / _FMA) and the VALU
 *                        screen read; 0: the index holds only the row-major
 *                        copy + the split-bf16 screen copy (2 N d 4 bytes
 *                        instead of 3), and scans that need the tiles return
 *                        LIRA_EUNSUPPORTED.  Read by the next add/build.
 *   LIRA_OPT_SCREEN      1: screened scan where supported (default); 0: always
 *                        the all-exact kernel
 *   LIRA_OPT_SPLIT       1: split-bf16 MFMA screen (default); 0: fp32 MFMA screen
 *   LIRA_OPT_QR          queries per screen work item: 0 auto (default), 64, 128; 32 (k > 56)
 *   LIRA_OPT_TWO_PHASE   nearest-probe group first: 1 auto (default), 0 off, 2 always
 *   LIRA_OPT_PRUNE       L2 triangle-inequality block skip / exact early abandon (1)
 *   LIRA_OPT_SEED        exact starting bound per query before the screen: 1 (default), 0 off
 *                        (2 / 3, the block-shared seed, were removed: LIRA_EUNSUPPORTED)
 *   LIRA_OPT_SHARE       per-block exchange of query bounds between work items (1)
 *   LIRA_OPT_ROUNDS      work items per workgroup target (0 = kernel default)
 *   LIRA_OPT_NEAR_ROUNDS the same for the nearest-probe group: 0 (default) auto -- the plan
 *                        picks 2..6 from the seed's estimate of the blocks the batch will screen; n fixed
 *   LIRA_OPT_MFMA        screen engine: 1 auto (default), 0 VALU, 2 MFMA wherever it fits
 *   LIRA_OPT_DEBUG       timing experiments only (results invalid): bit mask, see lira_screen.hip.
 *                        Production builds accept only 0 and return LIRA_EUNSUPPORTED otherwise;
 *                        a -DLIRA_DEBUG build (tools/build_variant.sh) accepts 0..255
 *   LIRA_OPT_PIPELINE, LIRA_OPT_RING, LIRA_OPT_WIDE
 *                        selected screen variants that measured slower than k_screen_m on every
 *                        config (k_screen_s, k_screen_w, k_screen_v) and were removed: 0 is
 *                        accepted (and read back), any other value returns LIRA_EUNSUPPORTED
 *   LIRA_OPT_PROBES_HINT expected valid probes per query when the probe lists are mostly -1
 *                        padding (a threshold selection padded to B): sizes the work split (0 = nprobe_max)
 *   LIRA_OPT_XHI         1: the split screen multiplies the query's hi + lo parts by x's hi part only
 *                        (half the staged bytes and MFMAs, a 2^-8 wider bound, more exact re-checks);
 *                        0: hi and lo; 2: hi parts of x and of the queries, 32 dims per MFMA
 *                        (k <= 24, else as 1; half the MFMAs again, bound + ||q - hi(q)|| (R + ..));
 *                        -1 (default): 2 for L2 (centred copy), 0 for IP
 *   LIRA_OPT_ORDER       (build time: set before lira_index_add_partitions) 1 (default, L2): store
 *                        each list's rows by ascending distance to the list's pivot, so tile radius
 *                        ranges are narrow and the triangle-inequality skip drops more; 0: list order.
 *                        Results never depend on it.
 *   LIRA_OPT_RSCREEN     1 (default): the wave-streaming screen k_screen_r where it applies (L2 or
 *                        centred IP on the split copy with the hi x hi screen, k <= 120, dpad <= 128
 *                        -- 2: also dpad > 128, a multiple of 64, the rows' hi parts streamed from
 *                        their records (measured slower than k_screen_m on GIST1M latent), the
 *                        per-query seed on, not PER_PARTITION): query rows' hi parts in LDS, each
 *                        wave streaming its own candidate tiles into registers; 0: k_screen_m
 *   LIRA_OPT_NEAR_FIRST  (k_screen_r) blocks of 256 candidates in the first chunk of every query
 *                        block's nearest partition: -1 (default) 4; 0: chunks of one size.  Those
 *                        small first chunks are queued first; the query block's later chunks wait
 *                        for its first one, so they start from the bounds it published instead of
 *                        the 128-row seed's.  Results never depend on it.
 *   LIRA_OPT_RESCAN      chunks whose screened list may have dropped a candidate (its 32nd key
 *                        within the final bound's reach) are scanned exactly again: -1 (default)
 *                        auto -- 1 where a chunk holds >= 8192 rows (32768 under k_screen_r, whose
 *                        spill lists leave few re-scans: BIGANN-size lists), else 0;
 *                        1: a pass that queues them, then k_rescan over all of them at once (a
 *                        wave per 64-row tile), whose exact survivors the merge takes; 0: inside
 *                        the merge, one wave per query.  Results never depend on it.
 *   LIRA_OPT_SPILL       (k_screen_r) records per query of its spill list -- the keys a full row
 *                        list evicts that the merge may still need, rechecked like list keys so
 *                        that no full list is re-scanned: -1 (default) 256; 0 none (full lists are
 *                        re-scanned as by k_screen_m); a query that overflows its records has its
 *                        full lists re-scanned instead.  Results never depend on it.
 *   LIRA_OPT_SEED_TILES  tiles of 64 rows of the nearest list the exact seed bound reads (fp32
 *                        tiles, L2, k <= 32): 0 (default) auto -- the seed fused with the
 *                        per-pair records (d <= 256): 4 below 4096 queries, else 2; the unfused
 *                        one: 1 for d > 512 (GIST1M), else 2; 1, 2 or 4 (fused only) fixed.
 *                        On the k_screen_r path the seed is k_seed_r (the first tiles screened on
 *                        the matrix cores, bound by the screen's error model; 4 tiles for k > 32).
 *                        Results never depend on it.  4 returns LIRA_EUNSUPPORTED where neither
 *                        fused seed can run (d > 256; IP uncentred or d > 128).
 *   LIRA_OPT_IP_CENTRE   (build time, IP indexes) 1 (default): like L2, store each list's rows
 *                        radius-ordered around its pivot c with the split copy of fl(x - c), so the
 *                        wave-streaming screen k_screen_r takes IP as q.x = q.fl(x - c) + q.c with a
 *                        Cauchy-Schwarz block skip (k <= 120, dpad <= 128); needs
 *                        LIRA_OPT_KEEP_TILES = 1 (the other screens read the fp32 tiles on such an
 *                        index).  0: the uncentred split copy (round-4 layout).  Results never
 *                        depend on it.
 *   LIRA_OPT_CHUNK       screen work items: at most this many blocks of 256 candidates per chunk
 *                        of a bucket (0, default: the plan's choice, <= 128).  Results never
 *                        depend on it.
 */
#define LIRA_OPT_KEEP_TILES 1
#define LIRA_OPT_SCREEN 2
#define LIRA_OPT_SPLIT 3
#define LIRA_OPT_QR 4
#define LIRA_OPT_TWO_PHASE 5
#define LIRA_OPT_PRUNE 6
#define LIRA_OPT_SEED 7
#define LIRA_OPT_SHARE 8
#define LIRA_OPT_ROUNDS 9
#define LIRA_OPT_NEAR_ROUNDS 10
#define LIRA_OPT_MFMA 11
#define LIRA_OPT_DEBUG 12
#define LIRA_OPT_PIPELINE 13
#define LIRA_OPT_RING 14
#define LIRA_OPT_PROBES_HINT 15
#define LIRA_OPT_XHI 16
#define LIRA_OPT_ORDER 17
#define LIRA_OPT_WIDE 18
#define LIRA_OPT_RSCREEN 19
#define LIRA_OPT_NEAR_FIRST 20
#define LIRA_OPT_RESCAN 21
#define LIRA_OPT_SPILL 22
#define LIRA_OPT_SEED_TILES 23
#define LIRA_OPT_IP_CENTRE 24
#define LIRA_OPT_CHUNK 25
int lira_index_set_option(lira_index *idx, int option, int64_t value);
int lira_index_get_option(const lira_index *idx, int option, int64_t *value);
/* 1 if the index holds the fp32 tile copy (LIRA_OPT_KEEP_TILES at build time) */
int lira_index_has_tiles(const lira_index *idx, int *out);

/* ------------------------------------------------- partition shards */
/*
 * k-way merge of per-shard top-k results: the exchange step of the
 * partition-sharded search (each rank holds the lists of its
 * own buckets, scans them for every query, and the ranks' (nq, k) results are
 * all-gathered and merged).  Each shard's lists hold a disjoint set of
 * (bucket, row) entries, so the k smallest keys of the union equal the
 * single-index result of search.cpp:495-514's top-k over all candidates.
 *   D, I      device (nparts, nq, k): fp32 / int64, each (nq, k) block in
 *             lira_scan_topk's output convention (sorted, -1 / +-inf pads)
 *   nparts    1..64 shards;  metric  LIRA_METRIC_L2 / _IP (the order)
 *   dedup     1: a gid reached through buckets of two shards is kept once
 *             (the scan's LIRA_SCAN_DEDUP across shards); 0: both kept
 *   out_D/I   device (nq, k), same convention.  Stream-ordered, capturable.
 */
int lira_merge_shards(const float *D, const int64_t *I, int64_t nparts, int64_t nq, int64_t k, int metric,
                      int dedup, float *out_D, int64_t *out_I, void *stream);

/* ----------------------------------------------------------- ranking */
/*
 * Query -> centroid Euclidean distances, exact fp32 in search.cpp's order:
 * out[q, b] = sqrt(sum_j (q_j - c_bj)^2), summed sequentially without FMA
 * (search.cpp:220-235); when scaler_mean/scaler_scale are non-NULL the result
 * is standardised in place: (d - mean_b) / (scale_b == 0 ? 1 : scale_b)
 * (search.cpp:238-250).  Replaces get_dist_cid (utils.py:98-118, scipy cdist)
 * for the query side.  q (nq,d), centroids (B,d), out (nq,B): device.
 */
int lira_centroid_dist(const float *q, int64_t nq, const float *centroids, int64_t n_centroids,
                       int64_t d, const float *scaler_mean, const float *scaler_scale,
                       float *out, void *stream);

/*
 * MFMA ranking GEMM (v_mfma_f32_32x32x2_f32): approximate squared distances
 * ||q||^2 + ||c||^2 - 2 q.c for every (q, b), out_sq (nq, B) device, plus a
 * per-query absolute error bound out_err (nq) such that
 * |out_sq - exact_sq| <= out_err for every b.  Feeds
 * lira_rank_nearest, which re-checks the nprobe boundary exactly.
 */
int lira_centroid_gemm(const float *q, int64_t nq, const float *centroids, int64_t n_centroids,
                       int64_t d, float *out_sq, float *out_err, void *stream);

/*
 * Fused IVF ranking: MFMA GEMM + exact boundary re-check.  Writes the nprobe
 * nearest centroids of every query, ordered by the exact search.cpp distance
 * sqrt(l2) ascending, ties -> smaller bucket id; identical to
 * lira_centroid_dist followed by lira_select_probes(NEAREST).  workspace:
 * device, at least lira_rank_workspace_size() bytes, or NULL to use the
 * handle-free internal path (allocates; not graph-capturable).
 */
int lira_rank_workspace_size(int64_t nq, int64_t n_centroids, size_t *bytes);
int lira_rank_nearest(const float *q, int64_t nq, const float *centroids, int64_t n_centroids,
                      int64_t d, int64_t nprobe, int32_t *out_probe, void *workspace,
                      size_t workspace_bytes, void *stream);

/*
 * Probe selection from an (n, B) score/distance matrix (device) into
 * out_probe (n, max_probe) int32 padded with -1, and out_nprobe (n) (nullable).
 *  NEAREST:       the max_probe smallest scores (ties -> smaller b), ascending.
 *  THRESHOLD_GE:  buckets with score >= thr in ascending b, argmax fallback
 *                 when none (first max wins) -- search.cpp:447-466.
 *  THRESHOLD_GT:  score > thr, no fallback -- LIRA_smallscale.py:206.
 * Threshold modes truncate at max_probe (pass max_probe = B for no truncation).
 * | LIRA_PROBE_BY_SCORE: threshold sets ordered by descending score (the scan
 * then meets each query's most probable partition first; same results).
 */
int lira_select_probes(const float *scores, int64_t n, int64_t n_centroids, int mode, float thr,
                       int64_t max_probe, int32_t *out_probe, int32_t *out_nprobe, void *stream);

/*
 * Reorder every row of a probe matrix (n, max_probe) int32, -1 padded, in place
 * by ascending key[i * n_centroids + b] (ties -> smaller b; -1 entries last):
 * the same probe SET, nearest partition first when key is the query ->
 * centroid distance.  No result of lira_scan_topk depends on the slot order,
 * but its speed does: slot 0 seeds the query's starting bound and forms the
 * nearest-probe group (a threshold selection in score order put an arbitrary
 * one of the probed partitions there; search.cpp:447-466 probes in bucket
 * order).  max_probe <= 256.  Stream-ordered, graph-capturable.
 */
int lira_order_probes(int32_t *probe, int64_t n, int64_t max_probe, const float *key, int64_t n_centroids,
                      void *stream);

/* -------------------------------------------------------------- scan */
/*
 * Batched candidate scan + exact top-k over the probed buckets.
 * Replaces search.cpp:468-514 (the per-query scan loop and nth_element top-k)
 * and the per-(query, bucket) faiss IndexFlat*.search calls of
 * get_cmp_recall (LIRA_smallscale.py:158-172).
 *   q          device fp32 (nq, d)
 *   probe      device int32 (nq, nprobe_max), -1 = unused slot
 *   k          1..256
 *   flags      LIRA_SCAN_DEDUP | LIRA_SCAN_PER_PARTITION | LIRA_SCAN_FMA | LIRA_SCAN_NO_PRUNE
 *   out_D      device fp32  (nq, k)  or (nq, nprobe_max, k) with PER_PARTITION
 *   out_I      device int64 (nq, k)  or (nq, nprobe_max, k) with PER_PARTITION
 *   out_ncand  device int64 (nq) or NULL: search.cpp's cmp_for_query
 *              (candidates scanned, replicas included, search.cpp:468-477)
 * Distances are bit-identical to search.cpp's sequential fp32 l2_sq / ip
 * (without LIRA_SCAN_FMA; with it, fma(q-x, q-x, acc) / fma(q, x, acc)).
 * Order: faiss convention -- L2 ascending squared distance, IP descending
 * inner product; ties -> smaller gid; pads (+inf, -1) for L2, (-inf, -1) IP.
 * workspace: device, >= lira_scan_workspace_size() bytes, or NULL to use a
 * buffer cached in the handle, grown on demand -- but never while `stream` is
 * being captured (LIRA_EINVAL: make one eager call of the same shape before the
 * capture); a cached buffer that a captured graph uses is kept allocated when a
 * later eager call outgrows it (until lira_index_destroy), so replays stay valid.
 *
 * Threading and streams.  Calls are asynchronous and stream-
 * ordered.  Several streams (and host threads) may search ONE handle at the same
 * time: the cached workspace is kept per stream (the plan counters, item tables,
 * row lists and bounds of one call are never shared with another stream's call),
 * and the host-side state (workspace table, profiling events, stats flags) is
 * guarded by a lock in the handle.  Up to 8 streams hold cached workspaces at
 * once; a 9th takes over the buffer of a stream whose last call has completed,
 * else the call returns LIRA_ESTATE (pass a workspace instead).  A capture on a
 * stream that has no buffer of its own (torch.cuda.graph's side stream) uses the
 * largest buffer an eager call sized: replay that graph on the stream whose eager
 * calls sized it (or pass a workspace), because the two share it.  Caller-supplied
 * workspaces are the caller's: one per concurrent call.  Not allowed concurrently
 * with a search: add_partitions / build / set_option / destroy on the same handle.
 * The work counters (lira_index_set_stats) and profiling sums aggregate every
 * stream's calls; lira_index_check reads one error word per handle.
 */
int lira_scan_workspace_size(const lira_index *idx, int64_t nq, int64_t nprobe_max, int64_t k,
                             unsigned flags, size_t *bytes);
int lira_scan_topk(lira_index *idx, const float *q, int64_t nq, const int32_t *probe,
                   int64_t nprobe_max, int64_t k, unsigned flags, float *out_D, int64_t *out_I,
                   int64_t *out_ncand, void *workspace, size_t workspace_bytes, void *stream);
/* the scan kernel (and its plan) lira_scan_topk would run for this shape, as
 * a NUL-terminated string into out (host, out_len bytes) -- for benchmarks */
int lira_scan_describe(const lira_index *idx, int64_t nq, int64_t nprobe_max, int64_t k, unsigned flags,
                       char *out, size_t out_len);

/*
 * Kernel timing for benchmarks.  While enabled, every lira_scan_topk records
 * HIP events on the caller's stream around its planning kernels, the k_scan
 * launch and the k_merge launch.  lira_index_profile_read synchronises on the
 * last recorded event, returns the summed milliseconds and the number of calls
 * since the previous read (or enable), and resets the sums.
 */
int lira_index_set_profiling(lira_index *idx, int enable);
int lira_index_profile_read(lira_index *idx, double *plan_ms, double *scan_ms, double *merge_ms,
                            int64_t *calls);

/*
 * Scan work counters, for measuring what the exact L2 pruning skips.  While
 * enabled, k_scan adds per candidate block (256 candidates x 32 query rows):
 *   [0] 16-dim wave-chunks computed, [1] wave-chunks a full scan computes
 *       (4 waves x dpad/16 per block, skipped blocks included),
 *   [2] blocks entered, [3] blocks dropped by the early abandon,
 *   [4] blocks skipped by the triangle-inequality test (never loaded),
 *   [5] candidates re-computed exactly by the screened path's merge,
 *   [6] chunks it re-scanned exactly (a screened list that may have dropped
 *       a needed candidate), [7] screened survivors appended to row lists.
 * The screened path (default) counts [0] as the (query row, candidate) pairs
 * it screened (padding rows included; x dpad = FMAs executed), and [2], [4],
 * [5], [6], [7]; there [1] = (query, partition) pairs the plan's partition
 * filter removed before any work item exists (the seed bound's triangle test
 * over the whole list) and [3] = their (query, candidate) pairs (never
 * screened).  The all-exact scan (LIRA_SCAN_EXACT) counts [0]..[4] as above.
 * lira_index_stats_read synchronises the device, copies the 8 sums to `out8`
 * (host) and resets them.  Costs a few atomics per block: keep it off when
 * timing.
 */
int lira_index_set_stats(lira_index *idx, int enable);
int lira_index_stats_read(lira_index *idx, uint64_t *out8);
/* which scan paths added to the counters since they were enabled or last read (call
 * it before lira_index_stats_read, which resets it): bit 0 the all-exact scan, bit 1
 * the screened one -- slots [1] and [3] mean different things on the two paths */
#define LIRA_STATS_PATH_EXACT 1
#define LIRA_STATS_PATH_SCREEN 2
int lira_index_stats_paths(const lira_index *idx, int *out);

/*
 * Device-side error word of the last scan/select on this handle (e.g. a probe
 * id >= n_lists, skipped): synchronises `stream`, returns LIRA_OK or LIRA_ERANGE
 * and clears the word.
 */
int lira_index_check(lira_index *idx, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LIRA_HIP_H */
