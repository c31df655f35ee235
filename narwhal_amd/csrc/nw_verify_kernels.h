// k_verify / k_slow_sig templates (one lane per signature).  Instantiated once per key comb window
// by nw_kv.hip (compiled with -DNW_WA=8/12/16/20, one object each, so the heavy kernels build in
// parallel); dispatched by launch_verify / launch_slow in nw_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "nw_point.h"
#include "nw_sha512.h"
#include "nw_chacha.h"
#include "nw_kernels.h"
#include "nw_core.h"

namespace nw {

// Signature i's inputs and h = SHA-512(R || A || M) mod l.
template <int MSGMODE>
__device__ __forceinline__ void lane_inputs(const VerifyParams& a, uint32_t i, uint32_t R[8], uint32_t S[8],
                                            uint32_t& slot, uint32_t& kinfo, uint32_t& cert, uint32_t h[8]) {
    uint32_t Aw[8];
    load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
    load_w8(S, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16 + 8);
    slot = a.signer[i];
    const bool in_cache = slot < a.nkeys;   // device inputs: an out-of-range slot is rejected
    slot = in_cache ? slot : 0u;
    load_w8(Aw, a.keys_raw + (size_t)slot * 8);
    kinfo = in_cache ? a.key_info[slot] : 0u;
    cert = a.sig_cert[i];
    if (MSGMODE == 0) {
        uint32_t M[8];
        load_w8(M, reinterpret_cast<const uint32_t*>(a.cert_msg) + (size_t)cert * 8);
        hram_msg32(h, R, Aw, M);
    } else {
        uint32_t hw[16];
        hram_generic(hw, R, Aw, a.msg_base + a.msg_off[i], a.msg_len[i]);
        sc_reduce512(h, hw);
    }
}

__device__ __forceinline__ void coeff_z(const VerifyParams& a, uint32_t i, uint32_t cert, uint32_t z4[4]) {
    const uint64_t bidx = a.cert_base + cert;
    chacha20_z(z4, a.zseed, i - a.cert_first[cert], (uint32_t)bidx, (uint32_t)(bidx >> 32), 0u);
}

// ------------------------------------------------------------------------------------ verify (P_i)
// One lane per signature: P_i = s_i B - h_i A_i, written as (X, Z) to pbuf with partial flags
// (S ok, A ok, A small, torsion coefficient for torsion keys).
// Occupancy: the 32-byte-digest kernel (certificates, votes, headers: the hot path) is held to
// 168 VGPRs = 3 waves per SIMD (a few spills, measured faster than 2 waves at 169-175 VGPRs).
// The generic-message kernel (worker chunks) is left unbounded: bounding it spills heavily.
#ifndef NW_DIG_LDS
#define NW_DIG_LDS 1   // digits precomputed into LDS (0: consumed from the scalar in the loop)
#endif
#ifndef NW_VERIFY_WAVES
#define NW_VERIFY_WAVES 3
#endif
template <int MSGMODE, int WA>
__global__ void __launch_bounds__(256, MSGMODE == 0 ? NW_VERIFY_WAVES : 1) k_verify(VerifyParams a) {
    const uint32_t gid = a.g0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= a.g0 + a.gn) return;
    // signer-grouped order: the 64 lanes of a wave mostly share one key table (TLB / cache locality)
    const uint32_t i = a.perm ? a.perm[gid] : gid;
    uint32_t R[8], S[8], h[8], slot, kinfo, cert;
    lane_inputs<MSGMODE>(a, i, R, S, slot, kinfo, cert, h);
    const bool sok = sc_is_canonical(S);
    const bool aok = (kinfo & KI_OK) != 0;
    uint32_t flags = (sok ? NW_F_S_OK : 0u) | (aok ? NW_F_A_OK : 0u) | ((kinfo & KI_SMALL) ? NW_F_A_SMALL : 0u);
    const uint32_t tk = (kinfo >> KI_TORSION_SHIFT) & 7u;
    if (a.batch_mode && tk != 0 && sok && aok) {   // torsion keys only (never for honest committees)
        uint32_t z4[4];
        coeff_z(a, i, cert, z4);
        flags |= torsion_coef(z4, h, tk) << NW_F_TCOEF_SHIFT;
    }
    uint32_t* frow = a.pbuf + (size_t)PREC_FLAGS_ROW * a.n;
    frow[gid] = flags;   // parked (coalesced) so neither flags nor i stays live through the combs
#if NW_DIG_LDS
    // every signed digit of s and h computed up front into LDS: neither scalar nor the digit carry
    // is live during the comb additions (register room for a three-product first group, NW_MADD3)
    constexpr int NB = comb_pos(B_WINDOW), NA = comb_pos(WA);
    __shared__ int digs[(NB + NA) * 256];
    {
        uint32_t sc[8];
        int carry = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) sc[k] = sok ? S[k] : 0u;
#pragma unroll
        for (int p = 0; p < NB; ++p) digs[p * 256 + threadIdx.x] = next_digit<B_WINDOW>(sc, carry);
        carry = 0;
#pragma unroll
        for (int p = 0; p < NA; ++p) digs[(NB + p) * 256 + threadIdx.x] = next_digit<WA>(h, carry);
    }
    ge_p3 P;
    comb_pass_dig<B_WINDOW, true, MSGMODE == 0 && NW_MADD_FUSED>(P, digs + threadIdx.x, 256, a.btab, false);
    comb_pass_dig<WA, false, MSGMODE == 0 && NW_MADD_FUSED>(P, digs + NB * 256 + threadIdx.x, 256,
                                                           a.key_tab + (size_t)slot * comb_words(WA), true);
#else
    // fused-carry products only in the 3-waves-per-SIMD kernel (MSGMODE 0); see ge_madd_s1
    const ge_p3 P = compute_P<WA, B_WINDOW, MSGMODE == 0 && NW_MADD_FUSED>(S, h, sok, a.btab,
                                                                           a.key_tab + (size_t)slot * comb_words(WA));
#endif
    // X, Z and the partial flags (y match, R sign, R small) in processing order, struct-of-arrays
    // (column gid): coalesced for k_finish, which completes the flags and writes flags[i].  R, i
    // and flags are re-read here rather than kept live through the combs (10 VGPRs): that keeps
    // the kernel at <= 168 VGPRs = 3 waves per SIMD.  The compiler barrier stops the re-reads from
    // being merged with the first loads.
    asm volatile("" ::: "memory");
    const uint32_t i2 = a.perm ? a.perm[gid] : gid;
    load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i2 * 16);
    store_prec_soa(a.pbuf, a.n, gid, P, verify_pflags(P, R, frow[gid]));
}

// Latency-mode kernel for small launches (nw_verify_split.h, compiled in nw_kvs.hip).
static constexpr uint32_t VERIFY_SPLIT_MAX_SIGS = 16384;
template <int WA>
hipError_t launch_split_wa(const VerifyParams& p, int msgmode, hipStream_t st);

// Exact path for signatures with D_i != O: Q_i = z_i (R_i - P_i); R decode failure -> F_R_BAD.
template <int MSGMODE, int WA>
__global__ void __launch_bounds__(256) k_slow_sig(VerifyParams a) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= *a.slow_count) return;
    const uint32_t i = a.slow_list[t];
    uint32_t* buf = a.slow_buf + (size_t)t * SLOW_WORDS;
    uint32_t R[8], S[8], h[8], slot, kinfo, cert;
    lane_inputs<MSGMODE>(a, i, R, S, slot, kinfo, cert, h);
    ge_p3 Rp;
    if (!ge_decompress(Rp, R)) {
        a.flags[i] |= NW_F_R_BAD;
        store_p3(buf, ge_identity());
        return;
    }
    const ge_p3 P = compute_P<WA>(S, h, true, a.btab, a.key_tab + (size_t)slot * comb_words(WA));
    uint32_t z4[4];
    coeff_z(a, i, cert, z4);
    store_p3(buf, slow_term(Rp, P, z4));
}

// Launch k_verify (slow = false, grid over p.gn) or k_slow_sig (slow = true, grid over n_upper).
template <int WA>
hipError_t launch_vs_wa(const VerifyParams& p, int msgmode, bool slow, uint32_t n_upper, hipStream_t st) {
    const dim3 b(256);
    const dim3 g(blocks_for(slow ? n_upper : p.gn, 256));
    if (!slow && p.gn <= VERIFY_SPLIT_MAX_SIGS) return launch_split_wa<WA>(p, msgmode, st);
    if (msgmode == 0) {
        if (slow) hipLaunchKernelGGL((k_slow_sig<0, WA>), g, b, 0, st, p);
        else hipLaunchKernelGGL((k_verify<0, WA>), g, b, 0, st, p);
    } else {
        if (slow) hipLaunchKernelGGL((k_slow_sig<1, WA>), g, b, 0, st, p);
        else hipLaunchKernelGGL((k_verify<1, WA>), g, b, 0, st, p);
    }
    return hipGetLastError();
}

}  // namespace nw
