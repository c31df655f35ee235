// Lone-wave inversion latency (one 64-lane wave alone on the GPU, shader cycles per inversion from
// s_memtime): 0 = fe_invert_var per lane (VALU), 1 = fe_invert_sg per lane (VALU, branch-free),
// 2 = fe_invert_wave (one inversion on wave-uniform operands: scalar unit), 3 = fe_invert_batched<1>
// (the wave's 64 values: butterfly + one scalar-unit inversion), 4 = <8> (8 groups of 8 lanes).
// Usage: tools/inv_lone [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../narwhal_amd/csrc/nw_inv.h"

using namespace nw;

__device__ fe seed_fe(uint32_t gid, uint32_t k) {
    fe f;
#pragma unroll
    for (int i = 0; i < 10; ++i) f.v[i] = ((gid * 2654435761u) ^ (k * 40503u + i * 977u)) & ((i & 1) ? M25 : M26);
    return f;
}

template <int MODE>
__global__ void __launch_bounds__(64) k_lone(unsigned long long* out, uint32_t* chk, int reps) {
    const uint32_t lane = threadIdx.x;
    fe x = seed_fe(MODE == 2 ? 0u : (MODE == 4 ? lane / 8 : lane), 1);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        fe y;
        if (MODE == 0) y = fe_invert_var(x);
        else if (MODE == 1) y = fe_invert_sg(x);
        else if (MODE == 2) y = fe_invert_wave(x);
        else if (MODE == 3) y = fe_invert_batched<1>(x);
        else y = fe_invert_batched<8>(x);
        x = fe_add(y, fe_one());   // the next input depends on this result
        x = fe_carry(x);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[0] = t1 - t0;
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) a ^= x.v[i];
    chk[lane] = a;
}

template <int MODE>
static double run(unsigned long long* d, uint32_t* c, int reps) {
    hipLaunchKernelGGL(k_lone<MODE>, dim3(1), dim3(64), 0, 0, d, c, 2);
    hipLaunchKernelGGL(k_lone<MODE>, dim3(1), dim3(64), 0, 0, d, c, reps);
    unsigned long long cyc = 0;
    if (hipMemcpy(&cyc, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (double)cyc / reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    unsigned long long* d;
    uint32_t* c;
    if (hipMalloc(&d, 8) != hipSuccess || hipMalloc(&c, 256) != hipSuccess) return 1;
    printf("cycles per inversion on a lone wave (s_memtime), %d chained inversions:\n", reps);
    printf("  per lane, variable-time (VALU):   %.0f\n", run<0>(d, c, reps));
    printf("  per lane, branch-free (VALU):     %.0f\n", run<1>(d, c, reps));
    printf("  one uniform value (SALU):         %.0f\n", run<2>(d, c, reps));
    printf("  batched over 64 lanes:            %.0f\n", run<3>(d, c, reps));
    printf("  batched over 8 groups of 8 lanes: %.0f\n", run<4>(d, c, reps));
    return 0;
}
