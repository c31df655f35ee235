// Placement probe for the lone SHA-512 chain: why does the same round-wave
// instruction stream take 9k cycles per block on some CUs and 16k on others?
//
// Every workgroup runs one two-lane round wave (nw_sha512_2l.h, K_t + W_t read from LDS with the
// shipped prefetch ring) over NB blocks, plus two companion waves whose behaviour is the variable:
//   mode 0: no companions (64-thread workgroup)
//   mode 1: companions only meet the round wave at one barrier per block
//   mode 2: companions run ~600 32-bit VALU instructions per block (less than the round wave's
//           ~1,700, so the round wave never waits at the barrier for them)
//   mode 3: companions write LDS rows between barriers (another buffer)
//   mode 4: companions load 128 B per lane from global memory between barriers
//   mode 5: companions run ~200 v_lshl_add_u64 per block
//   mode 6: companions run ~200 64-bit rotate-xor steps (v_alignbit_b32 + v_xor) per block
// The round wave also records the cycles it spends in the per-block barrier.
// G workgroups run at once; each records XCC_ID, HW_ID, its round wave's s_memtime cycles and
// s_memrealtime ticks, so one launch shows the spread over many CUs.
// Build: hipcc -O3 --offload-arch=gfx950 -I narwhal_amd/csrc tools/sha_place.hip -o tools/sha_place
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "nw_sha512.h"
#include "nw_sha512_2l.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

using namespace nw;

template <int MODE>
__global__ void __launch_bounds__(192) k_place(uint32_t nb, const uint64_t* kwin, const uint64_t* big, uint64_t* rec,
                                               uint64_t* sink) {
    __shared__ uint64_t kw[80][33];
    __shared__ uint64_t scratch[2][80][64];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const bool odd = lane & 1u;
    if (wave == 0) {
        for (uint32_t t = lane; t < 80 * 33; t += 64) kw[t / 33][t % 33] = (t % 33 == 32) ? 1ull : kwin[t / 33];
    }
    __syncthreads();
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        uint64_t h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = SHA512_IV[(odd ? 0 : 4) + k];
        Sha2L c;
        c.init(odd);
        const uint32_t col = odd ? 32u : (lane >> 1);
        const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
        uint64_t twait = 0;
        for (uint32_t b = 0; b < nb; ++b) {
            c.block(h, [&](int t) { return kw[t][col]; });
            if (MODE != 0) {
                const uint64_t tb = __builtin_amdgcn_s_memtime();
                __syncthreads();
                twait += __builtin_amdgcn_s_memtime() - tb;
            }
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            uint64_t* r = rec + (size_t)blockIdx.x * 8;
            r[0] = t1 - t0;
            r[1] = r1 - r0;
            r[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
            r[3] = __builtin_amdgcn_s_getreg((3 << 11) | 20);    // XCC_ID
            r[4] = h[0] ^ h[1] ^ h[2] ^ h[3];
            r[5] = twait;
        }
        return;
    }
    // companions
    uint64_t acc = lane + wave;
    const uint64_t* src = big + ((size_t)blockIdx.x * 2 + (wave - 1)) * (size_t)nb * 16 * 64;
    for (uint32_t b = 0; b < nb; ++b) {
        if (MODE == 2) {
            uint32_t a32 = (uint32_t)acc, b32 = (uint32_t)(acc >> 32);
#pragma unroll 8
            for (int k = 0; k < 200; ++k) {
                a32 = (a32 ^ (b32 << 3)) + (uint32_t)k;
                b32 = b32 ^ a32;
            }
            acc = ((uint64_t)b32 << 32) | a32;
        } else if (MODE == 5) {
#pragma unroll 8
            for (int k = 0; k < 200; ++k) {
                acc = acc + (acc << 1);
                asm volatile("" : "+v"(acc));
            }
        } else if (MODE == 6) {
#pragma unroll 8
            for (int k = 0; k < 200; ++k) acc = rotr64v(acc, 19) ^ (acc + k);
        } else if (MODE == 3) {
#pragma unroll
            for (int t = 0; t < 40; ++t) scratch[wave - 1][t + 40 * (b & 1)][lane] = acc + t;
        } else if (MODE == 4) {
            const uint4* q = reinterpret_cast<const uint4*>(src + (size_t)b * 16 * 64 + lane * 16);
            uint4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = q[j];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += v[j].x ^ v[j].w;
        }
        __syncthreads();
    }
    if (acc == 0x12345) sink[0] = acc;   // keeps the companions' work live
}

int main(int argc, char** argv) {
    const uint32_t nb = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
    const uint32_t G = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
    const int reps = argc > 3 ? atoi(argv[3]) : 2;
    std::vector<uint64_t> kw(80);
    for (int t = 0; t < 80; ++t) kw[t] = SHA512_K[t] ^ (0x9E3779B97F4A7C15ull * (t + 1));
    uint64_t *d_kw, *d_big, *d_rec, *d_sink;
    const size_t big_words = (size_t)G * 2 * nb * 16 * 64;
    CHECK(hipMalloc(&d_kw, 80 * 8));
    CHECK(hipMemcpy(d_kw, kw.data(), 80 * 8, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_big, big_words * 8));
    CHECK(hipMemset(d_big, 0x5A, big_words * 8));
    CHECK(hipMalloc(&d_rec, (size_t)G * 64));
    CHECK(hipMalloc(&d_sink, 64));
    std::vector<uint64_t> rec((size_t)G * 8);
    for (int mode = 0; mode <= 6; ++mode) {
        for (int rep = 0; rep < reps; ++rep) {
            const dim3 blk(mode == 0 ? 64 : 192);
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_place<0>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
                case 1: hipLaunchKernelGGL(k_place<1>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
                case 2: hipLaunchKernelGGL(k_place<2>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
                case 3: hipLaunchKernelGGL(k_place<3>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
                case 4: hipLaunchKernelGGL(k_place<4>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
                case 5: hipLaunchKernelGGL(k_place<5>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
                default: hipLaunchKernelGGL(k_place<6>, dim3(G), blk, 0, 0, nb, d_kw, d_big, d_rec, d_sink); break;
            }
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(rec.data(), d_rec, rec.size() * 8, hipMemcpyDeviceToHost));
            for (uint32_t g = 0; g < G; ++g) {
                const uint64_t* r = &rec[(size_t)g * 8];
                const uint32_t hw = (uint32_t)r[2];
                printf("{\"mode\": %d, \"rep\": %d, \"wg\": %u, \"xcc\": %u, \"se\": %u, \"sh\": %u, \"cu\": %u, \"simd\": %u, "
                       "\"cyc_per_block\": %.0f, \"wait_per_block\": %.0f, \"ns_per_block\": %.1f, \"ghz\": %.3f}\n",
                       mode, rep, g, (uint32_t)r[3] & 15u, (hw >> 13) & 7u, (hw >> 12) & 1u, (hw >> 8) & 15u,
                       (hw >> 4) & 3u, (double)r[0] / nb, (double)r[5] / nb, r[1] * 10.0 / nb, (double)r[0] / (r[1] * 10.0));
            }
        }
    }
    return 0;
}
