// Variant benchmark for the k_verify comb loop (developer tool).
// Builds real basepoint (w16) and 100 committee-key tables (w16) with the library's own table
// code, then times P = s B - h A over 1M random (s, h, signer) with several loop variants.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../narwhal_amd/csrc/nw_core.h"

using namespace nw;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int W>
__global__ void kprep(uint32_t nk, const uint32_t* raw, uint32_t* info, uint32_t* bases) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < nk) info[j] = key_prep_one<W>(raw + j * 8, bases + (size_t)j * comb_pos(W) * 40);
}
template <int W>
__global__ void kent(uint32_t nk, const uint32_t* bases, uint32_t* tab) {
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t per = (uint64_t)comb_pos(W) * comb_ent(W);
    if (g >= nk * per) return;
    uint32_t j = g / per, r = g % per;
    comb_entry_one<W>(bases + (size_t)j * comb_pos(W) * 40, r / comb_ent(W), r % comb_ent(W), tab + (size_t)j * comb_words(W));
}

// Variant 0: library loop (no prefetch)
template <int WA>
__global__ void __launch_bounds__(256) v0(uint32_t n, const uint32_t* sc, const uint32_t* slot, const uint32_t* btab,
                                          const uint32_t* ktab, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s[8], h[8];
    load_w8(s, sc + (size_t)i * 16);
    load_w8(h, sc + (size_t)i * 16 + 8);
    ge_p3 P = comb_sB_minus_hA<16, WA>(s, h, btab, ktab + (size_t)slot[i] * comb_words(WA));
    store_xyz(out + (size_t)i * 32, P);
}

// Variant 1: register prefetch of the next table entry (software pipelined gathers)
template <int W>
__device__ __forceinline__ void comb_pf(ge_p3& P, uint32_t sc[8], const uint32_t* tab, bool neg_pos) {
    int carry = 0;
    int d = next_digit<W>(sc, carry);
    const uint4* q = reinterpret_cast<const uint4*>(tab + (size_t)(d < 0 ? -d : d) * PRECOMP_WORDS);
    uint4 cur[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = q[k];
#pragma nounroll
    for (int pos = 0; pos < comb_pos(W); ++pos) {
        uint4 nxt[8];
        int dn = 0;
        if (pos + 1 < comb_pos(W)) {
            dn = next_digit<W>(sc, carry);
            const uint4* qn = reinterpret_cast<const uint4*>(
                tab + ((size_t)(pos + 1) * comb_ent(W) + (dn < 0 ? -dn : dn)) * PRECOMP_WORDS);
#pragma unroll
            for (int k = 0; k < 8; ++k) nxt[k] = qn[k];
        }
        uint32_t w[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            w[4 * k] = cur[k].x; w[4 * k + 1] = cur[k].y; w[4 * k + 2] = cur[k].z; w[4 * k + 3] = cur[k].w;
        }
        P = ge_madd(P, ge_precomp_cneg(ge_precomp_from_words(w), neg_pos ? d > 0 : d < 0));
#pragma unroll
        for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        d = dn;
    }
}

template <int WA>
__global__ void __launch_bounds__(256) v1(uint32_t n, const uint32_t* sc, const uint32_t* slot, const uint32_t* btab,
                                          const uint32_t* ktab, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s[8], h[8];
    load_w8(s, sc + (size_t)i * 16);
    load_w8(h, sc + (size_t)i * 16 + 8);
    ge_p3 P = ge_identity();
    comb_pf<16>(P, s, btab, false);
    comb_pf<WA>(P, h, ktab + (size_t)slot[i] * comb_words(WA), true);
    store_xyz(out + (size_t)i * 32, P);
}

// Variant 2: same as v0 but forced to 4 waves/SIMD (128 VGPR cap)
template <int WA>
__global__ void __launch_bounds__(256, 4) v2(uint32_t n, const uint32_t* sc, const uint32_t* slot, const uint32_t* btab,
                                             const uint32_t* ktab, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s[8], h[8];
    load_w8(s, sc + (size_t)i * 16);
    load_w8(h, sc + (size_t)i * 16 + 8);
    ge_p3 P = comb_sB_minus_hA<16, WA>(s, h, btab, ktab + (size_t)slot[i] * comb_words(WA));
    store_xyz(out + (size_t)i * 32, P);
}

// Variant 3: prefetch + 3 waves/SIMD cap
template <int WA>
__global__ void __launch_bounds__(256, 3) v3(uint32_t n, const uint32_t* sc, const uint32_t* slot, const uint32_t* btab,
                                             const uint32_t* ktab, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s[8], h[8];
    load_w8(s, sc + (size_t)i * 16);
    load_w8(h, sc + (size_t)i * 16 + 8);
    ge_p3 P = ge_identity();
    comb_pf<16>(P, s, btab, false);
    comb_pf<WA>(P, h, ktab + (size_t)slot[i] * comb_words(WA), true);
    store_xyz(out + (size_t)i * 32, P);
}

// Variant 4: all-L2 experiment: every signature uses slot 0 and the same digits (table hot in L2)
template <int WA>
__global__ void __launch_bounds__(256) v4(uint32_t n, const uint32_t* sc, const uint32_t* slot, const uint32_t* btab,
                                          const uint32_t* ktab, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s[8], h[8];
    load_w8(s, sc + (size_t)i * 16);
    load_w8(h, sc + (size_t)i * 16 + 8);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s[k] &= 0x00030003u;   // digits in {0..3}: the touched table lines stay hot in L1/L2
        h[k] &= 0x00030003u;
    }
    ge_p3 P = comb_sB_minus_hA<16, WA>(s, h, btab, ktab);
    store_xyz(out + (size_t)i * 32, P);
}

template <typename K>
float timeit(K kern, uint32_t n, const uint32_t* sc, const uint32_t* slot, const uint32_t* bt, const uint32_t* kt,
             uint32_t* out) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, n, sc, slot, bt, kt, out);
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, n, sc, slot, bt, kt, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

template <int W>
uint32_t* build_keys(const uint32_t* d_raw, uint32_t nk, uint32_t* d_info, uint32_t* d_bases) {
    uint32_t* t;
    CK(hipMalloc(&t, comb_words(W) * 4 * (size_t)nk));
    hipLaunchKernelGGL(kprep<W>, dim3((nk + 63) / 64), dim3(64), 0, 0, nk, d_raw, d_info, d_bases);
    hipLaunchKernelGGL(kent<W>, dim3((uint64_t(nk) * comb_pos(W) * comb_ent(W) + 255) / 256), dim3(256), 0, 0, nk, d_bases, t);
    CK(hipDeviceSynchronize());
    return t;
}

int main(int argc, char** argv) {
    const uint32_t n = 1000042, nk = 100;
    std::vector<uint8_t> raw(32 * (nk + 1));
    const uint8_t bas[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                             0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
    for (uint32_t k = 0; k <= nk; ++k) {
        for (int b = 0; b < 32; ++b) raw[32 * k + b] = bas[b];
        raw[32 * k] ^= (uint8_t)(k * 2);
    }
    uint32_t *d_raw, *d_info, *d_bases, *d_btab, *d_sc, *d_slot, *d_slot_sorted, *d_out;
    CK(hipMalloc(&d_raw, raw.size()));
    CK(hipMemcpy(d_raw, raw.data(), raw.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_info, 4 * (nk + 1)));
    CK(hipMalloc(&d_bases, (size_t)(nk + 1) * 32 * 40 * 4));
    d_btab = build_keys<16>(d_raw, 1, d_info, d_bases);
    uint32_t* k16 = build_keys<16>(d_raw + 8, nk, d_info, d_bases);
    uint32_t* k12 = build_keys<12>(d_raw + 8, nk, d_info, d_bases);
    uint32_t* k8 = build_keys<8>(d_raw + 8, nk, d_info, d_bases);
    std::vector<uint32_t> sc(16 * (size_t)n), slot(n), slot_sorted(n);
    srand(1);
    for (size_t i = 0; i < sc.size(); ++i) sc[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    for (uint32_t i = 0; i < n; ++i) {
        sc[16 * i + 7] &= 0x0FFFFFFF;
        sc[16 * i + 15] &= 0x0FFFFFFF;
        slot[i] = (uint32_t)(rand() % nk);
        slot_sorted[i] = (uint32_t)((uint64_t)i * nk / n);
    }
    CK(hipMalloc(&d_sc, sc.size() * 4));
    CK(hipMalloc(&d_slot, slot.size() * 4));
    CK(hipMalloc(&d_slot_sorted, slot.size() * 4));
    CK(hipMalloc(&d_out, (size_t)n * 32 * 4));
    CK(hipMemcpy(d_sc, sc.data(), sc.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_slot, slot.data(), slot.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_slot_sorted, slot_sorted.data(), slot.size() * 4, hipMemcpyHostToDevice));
    printf("{\"v0_lib_w16\": %.3f, \"v3_pf_w16\": %.3f, \"v3_pf_w16_sorted\": %.3f, \"v3_pf_w12\": %.3f, \"v3_pf_w12_sorted\": %.3f, "
           "\"v3_pf_w8\": %.3f, \"v4_hot_w16\": %.3f, \"v4_hot_w12\": %.3f, \"v0_lib_w8\": %.3f}\n",
           timeit(v0<16>, n, d_sc, d_slot, d_btab, k16, d_out), timeit(v3<16>, n, d_sc, d_slot, d_btab, k16, d_out),
           timeit(v3<16>, n, d_sc, d_slot_sorted, d_btab, k16, d_out), timeit(v3<12>, n, d_sc, d_slot, d_btab, k12, d_out),
           timeit(v3<12>, n, d_sc, d_slot_sorted, d_btab, k12, d_out), timeit(v3<8>, n, d_sc, d_slot, d_btab, k8, d_out),
           timeit(v4<16>, n, d_sc, d_slot, d_btab, k16, d_out), timeit(v4<12>, n, d_sc, d_slot, d_btab, k12, d_out),
           timeit(v0<8>, n, d_sc, d_slot, d_btab, k8, d_out));
    return 0;
}
