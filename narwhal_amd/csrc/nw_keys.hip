// Key-cache builders (decode + comb tables, once per committee) and the signing kernel
// (synthetic workloads / crypto::Signature::new).
#include <hip/hip_runtime.h>
#include "nw_point.h"
#include "nw_kernels.h"
#include "nw_core.h"

namespace nw {

// ------------------------------------------------------------------------------------ key cache
// One thread per key: decode, small-order flag, torsion index, comb bases 2^(W i) A.
template <int W>
__global__ void __launch_bounds__(64) k_key_prep(uint32_t nk, const uint32_t* keys_raw, uint32_t* key_info,
                                                 uint32_t* bases) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nk) return;
    key_info[j] = key_prep_one<W>(keys_raw + (size_t)j * 8, bases + (size_t)j * comb_pos(W) * 40);
}

// One thread per (key, position, chunk of COMB_CH entries): consecutive multiples with one batched
// inversion per chunk (comb_chunk_build).
static constexpr int COMB_CH = 8;

template <int W>
__global__ void __launch_bounds__(256) k_comb_build(uint32_t nk, const uint32_t* bases, uint32_t* tab,
                                                    size_t stride) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nch = (comb_ent(W) + COMB_CH - 1) / COMB_CH;
    const uint64_t per_key = (uint64_t)comb_pos(W) * nch;
    if (gid >= (uint64_t)nk * per_key) return;
    const uint32_t j = (uint32_t)(gid / per_key);
    const uint64_t rem = gid % per_key;
    comb_chunk_build<W, COMB_CH>(bases + (size_t)j * comb_pos(W) * 40, (uint32_t)(rem / nch), (uint32_t)(rem % nch),
                                 tab + (size_t)j * stride);
}

// The negated copy T- of each key's table, written right after it (tab + j * stride + comb_words(W)):
// entry e of T- is -T[e] = ((y-x)/2, (y+x)/2, -d x y), d x y carried to tight limbs.  k_verify then
// takes a signed digit's entry from T+ or T- by address, with no negation in the addition.
template <int W>
__global__ void __launch_bounds__(256) k_comb_negate(uint32_t nk, uint32_t* tab, size_t stride) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t per_key = (uint64_t)comb_pos(W) * comb_ent(W);
    if (gid >= (uint64_t)nk * per_key) return;
    const uint32_t* src = tab + (size_t)(gid / per_key) * stride + (size_t)(gid % per_key) * PRECOMP_WORDS;
    const ge_precomp q = ge_precomp_from_words(src);
    ge_precomp r;
    r.ypx = q.ymx;
    r.ymx = q.ypx;
    r.xy2d = fe_carry(fe_neg(q.xy2d));
    uint32_t w[PRECOMP_WORDS];
    precomp_to_words(r, w);
    uint4* dst = reinterpret_cast<uint4*>(const_cast<uint32_t*>(src) + comb_words(W));
#pragma unroll
    for (int k = 0; k < PRECOMP_WORDS / 4; ++k) dst[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

// ------------------------------------------------------------------------------------ signing
template <int MW>
__global__ void __launch_bounds__(256) k_sign(uint32_t n, const uint32_t* seeds, const uint32_t* msgs,
                                              const uint32_t* btab, uint32_t* pk_out, uint32_t* sig_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t pk[8], sig[16];
    sign_one<MW>(seeds + (size_t)i * 8, msgs + (size_t)i * MW, btab, pk, sig);
    if (pk_out) {
#pragma unroll
        for (int k = 0; k < 8; ++k) pk_out[(size_t)i * 8 + k] = pk[k];
    }
    if (sig_out) {
#pragma unroll
        for (int k = 0; k < 16; ++k) sig_out[(size_t)i * 16 + k] = sig[k];
    }
}

template <int W>
static hipError_t launch_key_prep_w(uint32_t nk, const uint32_t* keys_raw, uint32_t* key_info, uint32_t* bases,
                                    uint32_t* tab, size_t stride, bool negtab, hipStream_t st) {
    hipLaunchKernelGGL(k_key_prep<W>, dim3(blocks_for(nk, 64)), dim3(64), 0, st, nk, keys_raw, key_info, bases);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t total = (uint64_t)nk * comb_pos(W) * ((comb_ent(W) + COMB_CH - 1) / COMB_CH);
    hipLaunchKernelGGL(k_comb_build<W>, dim3(blocks_for(total, 256)), dim3(256), 0, st, nk, bases, tab, stride);
    e = hipGetLastError();
    if (e != hipSuccess || !negtab) return e;
    const uint64_t ents = (uint64_t)nk * comb_pos(W) * comb_ent(W);
    hipLaunchKernelGGL(k_comb_negate<W>, dim3(blocks_for(ents, 256)), dim3(256), 0, st, nk, tab, stride);
    return hipGetLastError();
}

hipError_t launch_key_prep(uint32_t nk, const uint32_t* keys_raw, uint32_t* key_info, uint32_t* bases,
                           uint32_t* tab, size_t stride, bool negtab, int window, hipStream_t st) {
    if (nk == 0) return hipSuccess;
    if (window < 8 || window > B_WINDOW || stride < comb_words(window) * (negtab ? 2 : 1)) return hipErrorInvalidValue;
    if (window == B_WINDOW) return launch_key_prep_w<B_WINDOW>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
    switch (window) {
        case 8: return launch_key_prep_w<8>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
        case 9: return launch_key_prep_w<9>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
        case 12: return launch_key_prep_w<12>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
        case 13: return launch_key_prep_w<13>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
        case 16: return launch_key_prep_w<16>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
        case 20: return launch_key_prep_w<20>(nk, keys_raw, key_info, bases, tab, stride, negtab, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_sign(uint32_t n, int msg_words, const uint32_t* seeds, const uint32_t* msgs,
                       const uint32_t* btab, uint32_t* pk, uint32_t* sig, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (msg_words == 8)
        hipLaunchKernelGGL(k_sign<8>, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, seeds, msgs, btab, pk, sig);
    else if (msg_words == 2)
        hipLaunchKernelGGL(k_sign<2>, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, seeds, msgs, btab, pk, sig);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace nw
