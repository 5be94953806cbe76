/*
 * sanitize_driver.c -- TEST INFRASTRUCTURE ONLY: runs every function of the
 * CPU oracle (lira_oracle.c, linked in) on one case read from a raw file, under
 * AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle sanitize`).
 * tests/test_oracle_sanitized.py writes the golden fixtures' inputs (and edge
 * cases) as such files, runs this program and compares its outputs bit for bit
 * with the fixtures' expected values -- the same checks as tests/test_oracle.py,
 * so an out-of-bounds read in the checker cannot hide a parity failure.
 *
 * usage: sanitize_driver <case.bin> <out.bin>
 * case.bin: int64 n, d, n_mul, nb, nq, nprobe, k, metric, dedup_rep, then
 *   x f32[n*d], d2b i32[n*n_mul], q f32[nq*d], probe i32[nq*nprobe],
 *   centroids f32[nb*d], mean f32[nb], scale f32[nb]
 * out.bin: int64 total, offsets i64[nb+1], ids i32[total], D f32[nq*k],
 *   I i64[nq*k], ncand i64[nq], Dp f32[nq*nprobe*k], Ip i64[nq*nprobe*k],
 *   qdist f32[nq*nb], qdist_std f32[nq*nb], probe_nearest i32[nq*nprobe],
 *   probe_ge i32[nq*nb], count_ge i32[nq], probe_gt i32[nq*nb], count_gt i32[nq]
 *   (the threshold selections run on qdist_std at thr 0)
 * Exit 0 on success; the sanitizers abort with a report on any error.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t oracle_build_csr(const int32_t *d2b, int64_t n, int64_t n_mul, int64_t nb, int64_t *offsets,
                         int32_t *ids);
void oracle_centroid_dist(const float *q, int64_t nq, const float *cent, int64_t nb, int64_t dim, float *out);
void oracle_standardize(float *dist, int64_t n, int64_t nb, const float *mean, const float *scale);
void oracle_probe_threshold(const float *scores, int64_t n, int64_t nb, float thr, int strict, int32_t *out,
                            int32_t *nprobe_out);
void oracle_probe_nearest(const float *dist, int64_t n, int64_t nb, int64_t nprobe, int32_t *out);
void oracle_scan_topk(const float *q, int64_t nq, int64_t dim, const int64_t *offsets, const int32_t *ids,
                      const float *vecs, const int32_t *probe, int64_t nprobe_max, int64_t k, int metric,
                      int dedup, float *out_D, int64_t *out_I, int64_t *ncand);
void oracle_scan_per_partition(const float *q, int64_t nq, int64_t dim, const int64_t *offsets,
                               const int32_t *ids, const float *vecs, const int32_t *probe,
                               int64_t nprobe_max, int64_t k, int metric, float *out_D, int64_t *out_I);

/* exact-size heap buffers, so ASan sees every overrun */
static void *take(FILE *f, size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (!p || (bytes && fread(p, 1, bytes, f) != bytes)) {
        fprintf(stderr, "short read (%zu bytes)\n", bytes);
        exit(2);
    }
    return p;
}

static void *alloc(size_t bytes) {
    void *p = malloc(bytes ? bytes : 1);
    if (!p) exit(3);
    memset(p, 0xA5, bytes);
    return p;
}

static void put(FILE *f, const void *p, size_t bytes) {
    if (bytes && fwrite(p, 1, bytes, f) != bytes) exit(4);
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s case.bin out.bin\n", argv[0]);
        return 1;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    int64_t h[9];
    if (fread(h, sizeof h, 1, f) != 1) return 2;
    const int64_t n = h[0], d = h[1], n_mul = h[2], nb = h[3], nq = h[4], np = h[5], k = h[6];
    const int metric = (int)h[7], rep = (int)h[8];
    float *x = take(f, sizeof(float) * n * d);
    int32_t *d2b = take(f, sizeof(int32_t) * n * n_mul);
    float *q = take(f, sizeof(float) * nq * d);
    int32_t *probe = take(f, sizeof(int32_t) * nq * np);
    float *cent = take(f, sizeof(float) * nb * d);
    float *mean = take(f, sizeof(float) * nb);
    float *scale = take(f, sizeof(float) * nb);
    fclose(f);

    int64_t *off = alloc(sizeof(int64_t) * (nb + 1));
    int32_t *ids_cap = alloc(sizeof(int32_t) * n * n_mul);
    const int64_t total = oracle_build_csr(d2b, n, n_mul, nb, off, ids_cap);
    if (total < 0) return 5;
    /* the lists' rows gathered into an exact-size copy (search.cpp:387-403) */
    int32_t *ids = alloc(sizeof(int32_t) * total);
    memcpy(ids, ids_cap, sizeof(int32_t) * total);
    free(ids_cap);
    float *vecs = alloc(sizeof(float) * total * d);
    for (int64_t r = 0; r < total; ++r) memcpy(vecs + r * d, x + (int64_t)ids[r] * d, sizeof(float) * d);

    float *D = alloc(sizeof(float) * nq * k);
    int64_t *I = alloc(sizeof(int64_t) * nq * k), *nc = alloc(sizeof(int64_t) * nq);
    oracle_scan_topk(q, nq, d, off, ids, vecs, probe, np, k, metric, rep, D, I, nc);
    float *Dp = alloc(sizeof(float) * nq * np * k);
    int64_t *Ip = alloc(sizeof(int64_t) * nq * np * k);
    oracle_scan_per_partition(q, nq, d, off, ids, vecs, probe, np, k, metric, Dp, Ip);
    float *qd = alloc(sizeof(float) * nq * nb), *qs = alloc(sizeof(float) * nq * nb);
    oracle_centroid_dist(q, nq, cent, nb, d, qd);
    memcpy(qs, qd, sizeof(float) * nq * nb);
    oracle_standardize(qs, nq, nb, mean, scale);
    int32_t *pn = alloc(sizeof(int32_t) * nq * np);
    oracle_probe_nearest(qd, nq, nb, np, pn);
    int32_t *pge = alloc(sizeof(int32_t) * nq * nb), *cge = alloc(sizeof(int32_t) * nq);
    int32_t *pgt = alloc(sizeof(int32_t) * nq * nb), *cgt = alloc(sizeof(int32_t) * nq);
    oracle_probe_threshold(qs, nq, nb, 0.0f, 0, pge, cge);
    oracle_probe_threshold(qs, nq, nb, 0.0f, 1, pgt, cgt);

    FILE *o = fopen(argv[2], "wb");
    if (!o) return 1;
    put(o, &total, sizeof total);
    put(o, off, sizeof(int64_t) * (nb + 1));
    put(o, ids, sizeof(int32_t) * total);
    put(o, D, sizeof(float) * nq * k);
    put(o, I, sizeof(int64_t) * nq * k);
    put(o, nc, sizeof(int64_t) * nq);
    put(o, Dp, sizeof(float) * nq * np * k);
    put(o, Ip, sizeof(int64_t) * nq * np * k);
    put(o, qd, sizeof(float) * nq * nb);
    put(o, qs, sizeof(float) * nq * nb);
    put(o, pn, sizeof(int32_t) * nq * np);
    put(o, pge, sizeof(int32_t) * nq * nb);
    put(o, cge, sizeof(int32_t) * nq);
    put(o, pgt, sizeof(int32_t) * nq * nb);
    put(o, cgt, sizeof(int32_t) * nq);
    fclose(o);
    free(x); free(d2b); free(q); free(probe); free(cent); free(mean); free(scale);
    free(off); free(ids); free(vecs); free(D); free(I); free(nc); free(Dp); free(Ip);
    free(qd); free(qs); free(pn); free(pge); free(cge); free(pgt); free(cgt);
    return 0;
}
