// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" entry points into the REFERENCE's own compiled search.cpp
// (/root/reference/search.cpp, built from its source by oracle/Makefile into
// oracle/_ref/libref_search.so).  Nothing here re-implements the reference:
// each wrapper only adapts plain pointers to the reference function's C++
// signature and calls the reference's code.  Used by tests to pin the oracle
// restatement (oracle/lira_oracle.c) against the reference's arithmetic.
//
// search.cpp needs cnpy::npy_load (cnpy.h:73), whose implementation is not
// vendored; it is only called from search.cpp's main(), which these tests
// never run, so the library is linked with that symbol left unresolved and is
// loaded lazily (RTLD_LAZY).  No stand-in for it exists anywhere.
#include <cstddef>
#include <vector>

// Prototypes of the reference functions (search.cpp:220-269).
void compute_l2_to_centroids(const float* query, const float* centroids, size_t n_bkt,
                             size_t dim, std::vector<float>& out_dist);
void standardize_distances(std::vector<float>& dist, const std::vector<float>& mean,
                           const std::vector<float>& scale);
float l2_sq(const float* a, const float* b, size_t dim);
float ip(const float* a, const float* b, size_t dim);

extern "C" {

float ref_l2_sq(const float* a, const float* b, long dim) { return l2_sq(a, b, (size_t)dim); }

float ref_ip(const float* a, const float* b, long dim) { return ip(a, b, (size_t)dim); }

// one query -> all centroids (search.cpp:220-235), then optional standardize (:238-250)
void ref_centroid_dist(const float* q, const float* cent, long nb, long dim, const float* mean,
                       const float* scale, float* out) {
    std::vector<float> d;
    compute_l2_to_centroids(q, cent, (size_t)nb, (size_t)dim, d);
    if (mean && scale) {
        std::vector<float> m(mean, mean + nb), s(scale, scale + nb);
        standardize_distances(d, m, s);
    }
    for (long i = 0; i < nb; ++i) out[i] = d[(size_t)i];
}

}  // extern "C"
