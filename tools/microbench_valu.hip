// Microbenchmark: fp32 VALU issue rate on gfx950 for plain vs packed adds,
// and for the scan's exact (q-x)^2 accumulate pattern, at 1..8 waves/SIMD.
// Build+run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/microbench_valu.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_IT 4096

__global__ void k_add(float *out, float x, int it) {
    float a[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = threadIdx.x * 1e-3f + i;
    for (int n = 0; n < it; ++n) {
#pragma unroll
        for (int i = 0; i < 32; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(x));
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += a[i];
    if (s == 1234.5f) out[0] = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_pkadd(float *out, float x, int it) {
    f2 a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
    f2 xx = {x, x};
    for (int n = 0; n < it; ++n) {
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(xx));
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i].x + a[i].y;
    if (s == 1234.5f) out[0] = s;
}

// the scan's inner pattern: 4 q x 8 x, acc += (q - x)^2, exact (no FMA)
__global__ void k_l2(float *out, float x0, int it) {
    float acc[4][8];
    float q[4], xv[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = threadIdx.x * 1e-3f + u;
#pragma unroll
    for (int v = 0; v < 8; ++v) xv[v] = x0 + v;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 8; ++v) acc[u][v] = 0;
    for (int n = 0; n < it; ++n) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                float d = q[u] - xv[v];
                acc[u][v] = acc[u][v] + d * d;
            }
#pragma unroll
        for (int v = 0; v < 8; ++v) asm volatile("" : "+v"(xv[v]));
    }
    float s = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 8; ++v) s += acc[u][v];
    if (s == 1234.5f) out[0] = s;
}

template <typename K>
static void run(const char *name, K kern, double ops_per_iter_per_lane, int wps) {
    float *out;
    hipMalloc(&out, 4);
    int cus = 256;
    dim3 grid(cus * wps), block(256);  // 4 waves per block = 1 per SIMD per block
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, grid, block, 0, 0, out, 1.0f, 16);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, grid, block, 0, 0, out, 1.0f, N_IT);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double lane_ops = ops_per_iter_per_lane * N_IT * grid.x * 256.0;
    printf("%-8s waves/SIMD=%d  %8.3f ms  %7.2f T lane-ops/s\n", name, wps, ms, lane_ops / ms / 1e9);
    hipFree(out);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run("add", k_add, 32, w);
        run("pk_add", k_pkadd, 32, w);
        run("l2_4x8", k_l2, 96, w);
    }
    return 0;
}
