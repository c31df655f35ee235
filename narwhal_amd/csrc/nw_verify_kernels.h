// k_verify / k_slow_prep templates (one lane per signature).  Instantiated once per key comb window
// by nw_kv.hip (compiled with -DNW_WA=8/12/16/20, one object each, so the heavy kernels build in
// parallel); dispatched by launch_verify / launch_slow in nw_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "nw_point.h"
#include "nw_sha512.h"
#include "nw_chacha.h"
#include "nw_kernels.h"
#include "nw_core.h"
#include "nw_quad.h"
#include "nw_cert.h"

namespace nw {

// Signature i's inputs and h = SHA-512(R || A || M) mod l.  cert is clamped to a valid index; the
// returned bool says the signature lies in no certificate's range (NO_CERT: it gets no verdict).
// PINFO (k_verify): the slot and certificate come from a.pinfo[gid] (processing order, coalesced) when
// the launch has one; else from a.signer[i] / a.sig_cert[i].
template <int MSGMODE, bool PINFO = false>
__device__ __forceinline__ bool lane_inputs(const VerifyParams& a, uint32_t i, uint32_t R[8], uint32_t S[8],
                                            uint32_t& slot, uint32_t& kinfo, uint32_t& cert, uint32_t h[8],
                                            uint32_t gid = 0) {
    uint32_t Aw[8];
    uint2 sc = make_uint2(0u, 0u);
    if (PINFO && a.pinfo) sc = a.pinfo[gid];
    load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
    load_w8(S, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16 + 8);
    slot = (PINFO && a.pinfo) ? sc.x : a.signer[i];
    const bool in_cache = slot < a.nkeys;   // device inputs: an out-of-range slot is rejected
    slot = in_cache ? slot : 0u;
    load_w8(Aw, a.keys_raw + (size_t)slot * 8);
    kinfo = in_cache ? a.key_info[slot] : 0u;
    cert = (PINFO && a.pinfo) ? sc.y : a.sig_cert[i];
    const bool nocert = cert == NO_CERT;   // a vote outside every range: k_finish gives it no verdict
    cert = nocert ? 0u : cert;
    if (MSGMODE == 0) {
        uint32_t M[8];
        load_w8(M, reinterpret_cast<const uint32_t*>(a.cert_msg) + (size_t)cert * 8);
        hram_msg32(h, R, Aw, M);
    } else {
        uint32_t hw[16];
        hram_generic(hw, R, Aw, a.msg_base + a.msg_off[i], a.msg_len[i]);
        sc_reduce512(h, hw);
    }
    return nocert;
}

// A signature whose y does not match R's (so D_i = R_i - P_i != O: it will take the exact batch
// path) parks its P_i for k_slow_prep, which would otherwise recompute h_i and both combs.  Rare:
// honest batches never take the branch.
// HAS_T false: P carries X, Y, Z only (k_verify's last addition skips T): parked rescaled.
template <bool HAS_T = true>
__device__ __forceinline__ uint32_t park_mismatch(const VerifyParams& a, uint32_t i, const ge_p3& P, uint32_t pf) {
    if (a.batch_mode && a.pslow && !(pf & PF_YMATCH) && (pf & (NW_F_S_OK | NW_F_A_OK)) == (NW_F_S_OK | NW_F_A_OK)) {
        if constexpr (HAS_T) store_p3(a.pslow + (size_t)i * 40, P);
        else store_p3(a.pslow + (size_t)i * 40, p3_from_xyz(P));
        pf |= NW_F_P_SAVED;
    }
    return pf;
}

// ------------------------------------------------------------------------------------ verify (P_i)
// One lane per signature: P_i = s_i B - h_i A_i, written as (X, Z) to pbuf with partial flags
// (S ok, A ok, A small, torsion coefficient for torsion keys).
// Occupancy: the 32-byte-digest kernel (certificates, votes, headers: the hot path) is held to
// 168 VGPRs = 3 waves per SIMD (a few spills, measured faster than 2 waves at 169-175 VGPRs).
// The generic-message kernel (worker chunks) is left unbounded: bounding it spills heavily.
#ifndef NW_VERIFY_WAVES
#define NW_VERIFY_WAVES 3
#endif
// NT: the key tables carry their negated copies (VerifyParams::key_negtab); the basepoint's does when
// B_NEGTAB.
template <int MSGMODE, int WA, bool NT>
__global__ void __launch_bounds__(256, MSGMODE == 0 ? NW_VERIFY_WAVES : 1) k_verify(VerifyParams a) {
    const uint32_t gid = a.g0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= a.g0 + a.gn) return;
    // signer-grouped order: the 64 lanes of a wave mostly share one key table (TLB / cache locality)
    const uint32_t i = a.perm ? a.perm[gid] : gid;
    uint32_t R[8], S[8], h[8], slot, kinfo, cert;
    const bool nocert = lane_inputs<MSGMODE, true>(a, i, R, S, slot, kinfo, cert, h, gid);
    const bool sok = sc_is_canonical(S);
    const bool aok = (kinfo & KI_OK) != 0;
    uint32_t flags = (sok ? NW_F_S_OK : 0u) | (aok ? NW_F_A_OK : 0u) | ((kinfo & KI_SMALL) ? NW_F_A_SMALL : 0u) |
                     (nocert ? PF_NOCERT : 0u);
    const uint32_t tk = (kinfo >> KI_TORSION_SHIFT) & 7u;
    if (a.batch_mode && tk != 0 && sok && aok) {   // torsion keys only (never for honest committees)
        uint32_t z4[4];
        coeff_z(a, i, cert, z4);
        flags |= torsion_coef(z4, h, tk) << NW_F_TCOEF_SHIFT;
    }
    uint32_t* frow = a.pbuf + (size_t)PREC_FLAGS_ROW * a.n;
    frow[gid] = flags;   // parked (coalesced) so neither flags nor i stays live through the combs
    // every signed digit of s and h computed up front into LDS: neither scalar nor the digit carry
    // is live during the comb additions (register room for a three-product first group, NW_MADD3)
    constexpr int NB = comb_pos(B_WINDOW), NA = comb_pos(WA);
    __shared__ int digs[(NB + NA) * 256];
    // R parked in LDS for the y-match after the combs (not live through them, and not re-read from
    // HBM: a scattered 32-B read that cost a line per signature; PMC cycles per C2 launch 2.04 ->
    // 2.01 M, profiles/r06/pmc_rsave_r06.txt)
    __shared__ uint32_t rsave[8 * 256];
#pragma unroll
    for (int k = 0; k < 8; ++k) rsave[k * 256 + threadIdx.x] = R[k];
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
    comb_pass_dig<B_WINDOW, true, MSGMODE == 0 && NW_MADD_FUSED, B_NEGTAB>(P, digs + threadIdx.x, 256, a.btab, false);
    comb_pass_dig<WA, false, MSGMODE == 0 && NW_MADD_FUSED, NT, true>(P, digs + NB * 256 + threadIdx.x, 256,
                                                               a.key_tab + (size_t)slot * a.key_stride, true);
    // X, Z and the partial flags (y match, R sign, R small) in processing order, struct-of-arrays
    // (column gid): coalesced for k_finish, which completes the flags and writes flags[i].  R (from
    // LDS), i and flags are re-read here rather than kept live through the combs (10 VGPRs): that
    // keeps the kernel at <= 168 VGPRs = 3 waves per SIMD.  The compiler barrier stops the re-reads
    // from being merged with the first loads.
    asm volatile("" ::: "memory");
    const uint32_t i2 = a.perm ? a.perm[gid] : gid;
#pragma unroll
    for (int k = 0; k < 8; ++k) R[k] = rsave[k * 256 + threadIdx.x];
    store_prec_soa(a.pbuf, a.n, gid, P, park_mismatch<false>(a, i2, P, verify_pflags(P, R, frow[gid])));
}

// Latency-mode kernel for small launches (nw_verify_split.h, compiled in nw_kvs.hip).
static constexpr uint32_t VERIFY_SPLIT_MAX_SIGS = 16384;
template <int WA>
hipError_t launch_split_wa(const VerifyParams& p, int msgmode, hipStream_t st);

// Exact path, step 1 (one lane per entry of the slow list, grid-stride): for a signature whose
// strict equation fails in a certificate not yet rejected, decode R (failure: F_R_BAD, and the
// certificate is rejected), form D_i = R_i - P_i and classify it:
//   SK_SMALL  8 D_i = O, or z_i = 0: then z_i D_i = (z_i mod 8) D_i, summed by k_cert_finalize;
//   SK_BIG    otherwise: z_i D_i has a nonzero prime-order component (0 < z_i < 2^128 < l).
// E = <B> (+) E[8] is a direct sum, so a certificate with exactly ONE SK_BIG entry cannot sum to the
// identity (its prime-order component is z_i D_i' != O) and is rejected without any scalar
// multiplication; only certificates with two or more SK_BIG entries need z_i D_i (k_slow_mul).
// Entries of certificates already rejected (bad S / undecodable A, from k_finish) are skipped.
// (bid, nb): this workgroup's index among the nb workgroups that share the list.
template <int MSGMODE, int WA>
__device__ __forceinline__ void slow_prep(const VerifyParams& a, uint32_t bid, uint32_t nb) {
    const uint32_t cnt = *a.slow_count;
    // Entries are dealt to the blocks first (entry t -> block t mod grid, thread t / grid): the few
    // thousand entries of an adversarial batch land on wave 0 of every block, one working wave per
    // CU, instead of filling the first blocks' four waves, which the dispatcher may pack two or three
    // to a SIMD (each entry is a long serial chain: sharing a SIMD stretched the kernel 3x,
    // measured at C5 with per-entry timestamps).  A wave with fewer entries than lanes runs
    // duplicate chains of its own entries on the idle lanes (no writes): a wave with a sparse EXEC
    // mask issues its chain up to 1.8x slower on some CUs.
    const uint32_t nthr = nb * blockDim.x;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t base = (threadIdx.x - lane) * nb + bid; base < cnt; base += nthr) {   // wave-uniform
        const uint32_t t_own = base + lane * nb;
        const uint32_t v = (uint32_t)__popcll(__ballot(t_own < cnt));   // entries of this wave: lanes [0, v)
        const bool owner = lane < v;
        const uint32_t t = owner ? t_own : base + (lane % v) * nb;
        const uint32_t i = a.slow_list[t];
        uint32_t* rec = a.slow_buf + (size_t)t * SLOW_WORDS;
        const uint32_t cert = a.sig_cert[i];   // slow-list entries always have an owner (k_finish)
        const uint32_t fi = a.flags[i];
        if (owner) a.flags[i] = fi & ~NW_F_P_SAVED;   // internal bit: never returned to the caller
        if (a.cert_state[cert] & CS_DOOM) {
            if (owner) rec[SLOW_KIND] = SK_SKIP;
            continue;
        }
        uint32_t R[8];
        load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
        ge_p3 Rp;
        if (!ge_decompress(Rp, R)) {
            if (owner) {
                a.flags[i] = (fi & ~NW_F_P_SAVED) | NW_F_R_BAD;
                atomicOr(&a.cert_state[cert], CS_RDOOM);
                rec[SLOW_KIND] = SK_SKIP;
            }
            continue;
        }
        ge_p3 P;
        if (fi & NW_F_P_SAVED) {
            P = load_p3(a.pslow + (size_t)i * 40);
        } else {   // y matched but x's sign did not (R = -P): recompute P
            uint32_t R2[8], S[8], h[8], slot, kinfo, c2;
            lane_inputs<MSGMODE>(a, i, R2, S, slot, kinfo, c2, h);
            P = compute_P<WA>(S, h, true, a.btab, a.key_tab + (size_t)slot * a.key_stride);
        }
        const ge_p3 D = ge_add(Rp, ge_cached_neg(ge_to_cached(P)));
        uint32_t z4[4];
        coeff_z(a, i, cert, z4);
        const bool zzero = (z4[0] | z4[1] | z4[2] | z4[3]) == 0;
        const ge_p3 D2 = ge_dbl(D), D4 = ge_dbl(D2);
        const bool small = ge_is_identity(ge_dbl(D4));
        const uint32_t kind = (small || zzero) ? SK_SMALL : SK_BIG;
        if (kind == SK_BIG) {
            if (owner) {
                atomicAdd(&a.cert_state[cert], 1u);
                store_p3(rec, D);
            }
        } else {
            // the term itself: z_i D_i = (z_i mod 8) D_i from D, 2D, 4D (k_cert_exact only adds records)
            const uint32_t z8 = zzero ? 0u : (z4[0] & 7u);
            ge_p3 t8 = ge_select(ge_identity(), D, (z8 & 1u) != 0);
            t8 = ge_add(t8, ge_to_cached(ge_select(ge_identity(), D2, (z8 & 2u) != 0)));
            t8 = ge_add(t8, ge_to_cached(ge_select(ge_identity(), D4, (z8 & 4u) != 0)));
            if (owner) store_p3(rec, t8);
        }
        if (owner) rec[SLOW_KIND] = kind;
    }
}

template <int MSGMODE, int WA>
__global__ void __launch_bounds__(256) k_slow_prep(VerifyParams a) {
    slow_prep<MSGMODE, WA>(a, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------ exact path, step 2
// z_i D_i for the SK_BIG entries of certificates that have two or more of them (the only case the
// direct-sum argument of k_slow_prep cannot decide): one quad per entry, every point operation
// split over the quad's 4 lanes (nw_quad.h), signed radix-16 digits of the 128-bit z_i with the
// multiples 1..8 D_i in LDS: 7 table operations + 128 doublings + 32 additions on the quad.
// 256-thread workgroups (64 quads) with the entries dealt to the blocks first: an adversarial
// batch's few hundred entries land on wave 0 of every block, one working wave per CU (one-wave
// blocks were packed up to three to a SIMD by the dispatcher, stretching the serial chains).
static constexpr uint32_t SLOW_MUL_QUADS = 64;   // per 256-thread workgroup
__device__ __forceinline__ void slow_mul(const VerifyParams& a, uint32_t bid, uint32_t nb, uint32_t (*tab)[8][40]) {
    const uint32_t cnt = *a.slow_count;
    const uint32_t qd = threadIdx.x >> 2, q = threadIdx.x & 3u;
    uint32_t (*T)[40] = tab[qd];
    // entries dealt to the blocks first (one wave each), as in k_slow_prep: a wave's time is one
    // chain whatever its number of quads, so spreading the entries keeps the waves short and apart.
    // A wave with fewer entries than quads runs duplicate chains of its own entries on the idle
    // quads (own LDS table slot, no record writes), so its EXEC mask stays full.
    const uint32_t wq = (threadIdx.x & 63u) >> 2;                    // quad index inside the wave
    for (uint32_t base = (qd - wq) * nb + bid; base < cnt; base += nb * SLOW_MUL_QUADS) {
        const uint32_t t_own = base + wq * nb;
        const uint32_t v = (uint32_t)__popcll(__ballot(t_own < cnt)) >> 2;   // entries of this wave: quads [0, v)
        const bool owner = wq < v;
        const uint32_t t = owner ? t_own : base + (wq % v) * nb;
        uint32_t* rec = a.slow_buf + (size_t)t * SLOW_WORDS;
        if (rec[SLOW_KIND] != SK_BIG) continue;                      // uniform over the quad
        const uint32_t i = a.slow_list[t];
        const uint32_t cert = a.sig_cert[i];
        const uint32_t cs = a.cert_state[cert];
        if ((cs & (CS_DOOM | CS_RDOOM)) || (cs & CS_BIG_MASK) < 2u) continue;
        const ge_p3 D = ge_to_vgpr(load_p3(rec));
        uint32_t z4[4];
        coeff_z(a, i, cert, z4);
        // T[k] = (k + 1) D
        ge_p3 m = D;
        if (q == 0) store_p3(T[0], m);
        m = ge_dbl_quad(D);
        if (q == 0) store_p3(T[1], m);
#pragma nounroll
        for (int k = 2; k < 8; ++k) {
            m = ge_add_quad(m, D);
            if (q == 0) store_p3(T[k], m);
        }
        __builtin_amdgcn_wave_barrier();
        // signed radix-16 digits d_0..d_31 in [-8, 8) plus a top carry d_32 in {0, 1}, packed as
        // nibbles with d_31 in the top nibble so the Horner loop shifts them out from the top
        uint32_t pk[4] = {0u, 0u, 0u, 0u};
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t b = ((z4[j >> 3] >> (4 * (j & 7))) & 15u) + carry;
            carry = b >= 8u ? 1u : 0u;
            pk[j >> 3] |= ((b - 16u * carry) & 15u) << (4 * (j & 7));
        }
        ge_p3 acc = ge_select(ge_to_vgpr(ge_identity()), D, carry != 0);
#pragma nounroll
        for (int j = 31; j >= 0; --j) {
            acc = ge_dbl_quad(ge_dbl_quad(ge_dbl_quad(ge_dbl_quad(acc))));
            const int d = (int)(pk[3] << 0) >> 28;                  // top nibble, sign-extended
#pragma unroll
            for (int w = 3; w > 0; --w) pk[w] = (pk[w] << 4) | (pk[w - 1] >> 28);
            pk[0] <<= 4;
            if (d != 0) {
                const ge_p3 e = load_p3(T[(d < 0 ? -d : d) - 1]);
                acc = ge_add_quad(acc, d < 0 ? ge_neg(e) : e);
            }
        }
        if (q == 0 && owner) {
            store_p3(rec, acc);
            rec[SLOW_KIND] = SK_MUL;
        }
        __builtin_amdgcn_wave_barrier();   // the table slot is rewritten by this quad's next entry
    }
}

// The whole exact path of a small call (at most SLOW_TAIL_MAX_SIGS signatures and TAIL_MAX_CERTS
// certificates: one header, one vote batch) in ONE workgroup: k_slow_prep, k_slow_mul and
// k_cert_tail as three phases with a workgroup barrier between them, one launch instead of three
// (~4-5 us of dispatch each, the whole cost when the slow list is empty).  Phase 1 gives every
// entry a lane of its own (256 >= nsigs); phase 2 runs 64 quads per pass; phase 3 is wave 0's.
template <int MSGMODE, int WA>
__global__ void __launch_bounds__(256) k_slow_tail(VerifyParams a, FinalizeParams f) {
    __shared__ uint32_t tab[SLOW_MUL_QUADS][8][40];
    slow_prep<MSGMODE, WA>(a, 0u, 1u);
    __threadfence();
    __syncthreads();
    slow_mul(a, 0u, 1u, tab);
    __threadfence();
    __syncthreads();   // tab is free again: phase 3 reuses it for its partial sums
    if (threadIdx.x >= 64) return;
    cert_tail(f, threadIdx.x, reinterpret_cast<uint32_t (*)[40]>(&tab[0][0][0]));
}

// Launch k_verify (slow = false, grid over p.gn) or k_slow_prep (slow = true: a grid-stride grid
// capped at one 256-thread block per CU, so an honest batch's empty exact path costs one small
// dispatch whatever n_upper is).
static constexpr uint32_t SLOW_MAX_BLOCKS = 256;
template <int WA>
hipError_t launch_vs_wa(const VerifyParams& p, int msgmode, bool slow, uint32_t n_upper, hipStream_t st) {
    const dim3 b(256);
    uint32_t nb = blocks_for(slow ? n_upper : p.gn, 256);
    if (slow && nb > SLOW_MAX_BLOCKS) nb = SLOW_MAX_BLOCKS;
    const dim3 g(nb);
    if (!slow && p.gn <= VERIFY_SPLIT_MAX_SIGS) return launch_split_wa<WA>(p, msgmode, st);
    if (msgmode == 0) {
        if (slow) hipLaunchKernelGGL((k_slow_prep<0, WA>), g, b, 0, st, p);
        else if (p.key_negtab) hipLaunchKernelGGL((k_verify<0, WA, true>), g, b, 0, st, p);
        else hipLaunchKernelGGL((k_verify<0, WA, false>), g, b, 0, st, p);
    } else {
        if (slow) hipLaunchKernelGGL((k_slow_prep<1, WA>), g, b, 0, st, p);
        else if (p.key_negtab) hipLaunchKernelGGL((k_verify<1, WA, true>), g, b, 0, st, p);
        else hipLaunchKernelGGL((k_verify<1, WA, false>), g, b, 0, st, p);
    }
    return hipGetLastError();
}

template <int WA>
hipError_t launch_slow_tail_wa(const VerifyParams& p, const FinalizeParams& f, int msgmode, hipStream_t st) {
    if (!slow_tail_fits(f.ncerts, f.nsigs)) return hipErrorInvalidValue;
    if (msgmode == 0) hipLaunchKernelGGL((k_slow_tail<0, WA>), dim3(1), dim3(256), 0, st, p, f);
    else hipLaunchKernelGGL((k_slow_tail<1, WA>), dim3(1), dim3(256), 0, st, p, f);
    return hipGetLastError();
}

}  // namespace nw
