// Microbenchmark: field inversion (Fermat chain vs safegcd divsteps) and field-multiplication
// throughput on gfx950, with every lane working on its own data (no memory traffic in the loop).
// Build: hipcc -O3 --offload-arch=gfx950 tools/inv_bench.hip -o tools/inv_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../narwhal_amd/csrc/nw_inv.h"

using namespace nw;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

__device__ fe seed_fe(uint32_t gid, uint32_t k) {
    fe f;
#pragma unroll
    for (int i = 0; i < 10; ++i) f.v[i] = ((gid * 2654435761u) ^ (k * 40503u + i * 977u)) & ((i & 1) ? M25 : M26);
    return f;
}

template <int MODE>
__global__ void __launch_bounds__(256) k_inv(uint32_t* out, int reps) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    fe x = seed_fe(gid, 1);
    for (int r = 0; r < reps; ++r) x = MODE == 0 ? fe_invert(x) : fe_invert_sg(x);
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) a ^= x.v[i];
    out[gid] = a;
}

// 4 independent chains of multiplications (ILP like a mixed addition's products)
__global__ void __launch_bounds__(256) k_mul(uint32_t* out, int reps) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    fe a = seed_fe(gid, 1), b = seed_fe(gid, 2), c = seed_fe(gid, 3), d = seed_fe(gid, 4);
    const fe m = seed_fe(gid, 5);
    for (int r = 0; r < reps; ++r) {
        a = fe_mul(a, m);
        b = fe_mul(b, m);
        c = fe_mul(c, m);
        d = fe_mul(d, m);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) s ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
    out[gid] = s;
}

__global__ void __launch_bounds__(256) k_sq(uint32_t* out, int reps) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    fe a = seed_fe(gid, 1), b = seed_fe(gid, 2), c = seed_fe(gid, 3), d = seed_fe(gid, 4);
    for (int r = 0; r < reps; ++r) {
        a = fe_sq(a);
        b = fe_sq(b);
        c = fe_sq(c);
        d = fe_sq(d);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) s ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
    out[gid] = s;
}

template <typename K>
static float time_kernel(K k, int blocks, uint32_t* buf, int reps) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, reps);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, reps);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t* buf;
    CHECK(hipMalloc(&buf, (size_t)cus * 16 * 256 * 4));
    for (int wps : {1, 2, 4}) {   // waves per SIMD (4 waves per block, `wps` blocks per CU)
        const int blocks = cus * wps;
        const double lanes = (double)blocks * 256;
        float ms0 = time_kernel(k_inv<0>, blocks, buf, 4);
        float ms1 = time_kernel(k_inv<1>, blocks, buf, 4);
        printf("{\"kernel\": \"invert\", \"waves_per_simd\": %d, \"fermat_us_per_inv_chain\": %.2f, "
               "\"safegcd_us_per_inv_chain\": %.2f, \"fermat_Minv_per_s\": %.1f, \"safegcd_Minv_per_s\": %.1f}\n",
               wps, ms0 * 1e3 / 4, ms1 * 1e3 / 4, lanes * 4 / (ms0 * 1e3), lanes * 4 / (ms1 * 1e3));
        float msm = time_kernel(k_mul, blocks, buf, 256);
        float mss = time_kernel(k_sq, blocks, buf, 256);
        printf("{\"kernel\": \"fe_mul/fe_sq\", \"waves_per_simd\": %d, \"Gmul_per_s\": %.1f, \"Gsq_per_s\": %.1f}\n", wps,
               lanes * 1024 / (msm * 1e6), lanes * 1024 / (mss * 1e6));
        fflush(stdout);
    }
    return 0;
}
