// Wave -> SIMD placement probe (digest packing): each wave of a 384-thread
// workgroup holding 126,720 B of LDS (+ a dynamic pad) writes its HW_ID; the host prints, per
// workgroup, the SIMD and CU of waves 0..5.  Usage: tools/wave_place [blocks] [pad_bytes] [spin_us]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(384) k_place(unsigned* out, unsigned spin) {
    __shared__ unsigned lds[126720 / 4];
    const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin * 100ull) {}
    if (lane == 0) out[blockIdx.x * 8 + w] = __builtin_amdgcn_s_getreg((31 << 11) | 4) + (lds[w] & 0u);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 20;
    const int pad = argc > 2 ? atoi(argv[2]) : 16000;
    const unsigned spin = argc > 3 ? (unsigned)atoi(argv[3]) : 2000;
    unsigned* d;
    if (hipMalloc(&d, blocks * 8 * 4) != hipSuccess) return 1;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_place), hipFuncAttributeMaxDynamicSharedMemorySize, pad) !=
        hipSuccess)
        return 2;
    hipLaunchKernelGGL(k_place, dim3(blocks), dim3(384), pad, 0, d, spin);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<unsigned> h(blocks * 8);
    if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 4;
    for (int b = 0; b < blocks; ++b) {
        printf("wg %2d:", b);
        for (int w = 0; w < 6; ++w) {
            const unsigned x = h[b * 8 + w];
            printf("  w%d simd%u cu%2u se%u wave%u", w, (x >> 4) & 3u, (x >> 8) & 15u, (x >> 13) & 7u, x & 15u);
        }
        printf("\n");
    }
    return 0;
}
