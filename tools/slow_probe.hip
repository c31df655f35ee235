// Lone-wave cost of the serial chains on the exact batch path and the latency path: how many
// shader cycles one wave spends on each building block, with all 64 lanes busy on independent data
// and with only the first 4 or 1 lanes active (the EXEC mask of k_slow_mul's quad / k_slow_prep's
// lane / k_finish's single inversion), over 8 launches each (different CUs).
// One workgroup of 64 threads per variant; s_memtime around the timed region.
//   fe_sq x254         the square-root / inversion exponent chain (fe_pow22523 is 250 + 11)
//   fe_mul x100        generic product
//   ge_decompress      R decompression (k_slow_prep, k_msm_prep)
//   ge_dbl x128        one-lane doublings
//   ge_dbl_quad x128   quad-split doublings (k_slow_mul, k_msm_final)
//   fe_invert_var      variable-time safegcd (k_finish for few signatures per lane)
//   fe_invert_sg       constant-time safegcd
// Build: hipcc -O3 --offload-arch=gfx950 -I narwhal_amd/csrc tools/slow_probe.hip -o tools/slow_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "nw_point.h"
#include "nw_quad.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

using namespace nw;

__device__ fe fe_seed(uint32_t s) {
    fe f;
#pragma unroll
    for (int k = 0; k < 10; ++k) f.v[k] = (s * 2654435761u + 97u * k) & ((k & 1) ? 0x1FFFFFFu : 0x3FFFFFFu);
    return f;
}

// lane-dependent (hence VGPR-resident) extended point; not on the curve, same arithmetic cost
__device__ ge_p3 ge_to_vgpr_probe(const fe& f) {
    ge_p3 p;
    p.X = f;
    p.Y = fe_seed(threadIdx.x * 3 + 5);
    p.Z = fe_one();
    p.T = fe_mul(p.X, p.Y);
    return p;
}

__device__ void sink(uint32_t* out, const fe& f) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) x ^= f.v[k];
    out[threadIdx.x] = x;
}

template <int V>
__global__ void __launch_bounds__(64) k_probe(uint32_t* out, uint64_t* cyc, uint32_t salt, uint32_t act) {
    fe f = fe_seed(threadIdx.x + salt);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x < act) {
    if (V == 0) {
        f = fe_sqn(f, 254);
        sink(out, f);
    } else if (V == 1) {
        fe g = fe_seed(threadIdx.x * 7 + salt);
#pragma nounroll
        for (int i = 0; i < 100; ++i) f = fe_mul(f, g);
        sink(out, f);
    } else if (V == 2) {
        uint32_t w[8];
        fe_tobytes_w(w, f);
        ge_p3 p;
        const bool ok = ge_decompress(p, w);
        sink(out, p.X);
        if (ok) out[64 + threadIdx.x] = 1;
    } else if (V == 3) {
        ge_p3 p = ge_to_vgpr_probe(f);
#pragma nounroll
        for (int i = 0; i < 128; ++i) p = ge_dbl(p);
        sink(out, p.X);
    } else if (V == 4) {
        ge_p3 p = ge_to_vgpr_probe(f);
#pragma nounroll
        for (int i = 0; i < 128; ++i) p = ge_dbl_quad(p);
        sink(out, p.X);
    } else if (V == 5) {
        sink(out, fe_invert_var(f));
    } else {
        sink(out, fe_invert_sg(f));
    }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        cyc[2 * V] = t1 - t0;
        cyc[2 * V + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
}

int main() {
    uint32_t* d_out;
    uint64_t* d_cyc;
    CHECK(hipMalloc(&d_out, 4096));
    const char* names[7] = {"fe_sq_x254", "fe_mul_x100", "ge_decompress", "ge_dbl_x128", "ge_dbl_quad_x128",
                            "fe_invert_var", "fe_invert_sg"};
    CHECK(hipMalloc(&d_cyc, 256));
    const uint32_t acts[3] = {64, 4, 1};
    for (int a = 0; a < 3; ++a) {
        for (int rep = 0; rep < 8; ++rep) {
            const uint32_t act = acts[a];
            hipLaunchKernelGGL(k_probe<0>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            hipLaunchKernelGGL(k_probe<1>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            hipLaunchKernelGGL(k_probe<2>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            hipLaunchKernelGGL(k_probe<3>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            hipLaunchKernelGGL(k_probe<4>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            hipLaunchKernelGGL(k_probe<5>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            hipLaunchKernelGGL(k_probe<6>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, rep, act);
            CHECK(hipDeviceSynchronize());
            uint64_t cyc[16];
            CHECK(hipMemcpy(cyc, d_cyc, 128, hipMemcpyDeviceToHost));
            for (int v = 0; v < 7; ++v)
                printf("{\"probe\": \"%s\", \"active_lanes\": %u, \"rep\": %d, \"cycles\": %llu, \"cu\": %u}\n",
                       names[v], act, rep, (unsigned long long)cyc[2 * v], (uint32_t)(cyc[2 * v + 1] >> 8) & 15u);
        }
    }
    return 0;
}
