// Latency-mode k_verify (k_verify_split) for small launches; compiled once per key window in
// nw_kvs.hip (a separate object from nw_kv.hip so the two heavy halves build in parallel).
#pragma once
#include "nw_verify_kernels.h"

namespace nw {

// ------------------------------------------------------------------------------------ latency mode
// Small launches (a single certificate, a vote batch: fewer signatures than the chip has SIMD
// lanes / VERIFY_SPLIT) leave most SIMDs idle and run each wave alone, at the lone-wave issue rate,
// so k_verify's time is the length of ONE signature's comb chain.  Here VERIFY_SPLIT lanes share a
// signature: the NPOS = comb_pos(WB) + comb_pos(WA) positions of its two combs are cut into
// contiguous blocks, each lane sums its block, and two shuffle levels add the partial points.
// Digits are taken from k' = k + sum_p 2^(W-1) 2^(W p) (signed radix-2^W digit p = window p of k'
// minus 2^(W-1)), so any lane can start at any position without the serial carry chain.  The
// output record is the one k_verify writes, for the same k_finish.
// 8 lanes per signature: ceil(NPOS / 8) mixed additions per lane (3 at W20) + 3 shuffle levels of
// full additions = 6 dependent point operations (~51 field products) against 6 + 2 (~62) with 4
// lanes; 16 lanes would be 2 + 4 (~54).
static constexpr int VERIFY_SPLIT = 8;
// VERIFY_SPLIT_MAX_SIGS (nw_verify_kernels.h): the split grid is then <= two waves per SIMD
// (1,024 SIMDs x 64 lanes x 2 / VERIFY_SPLIT)
static_assert(VERIFY_SPLIT_MAX_SIGS * VERIFY_SPLIT <= 2 * 256 * 4 * 64, "split grid larger than two waves per SIMD");
static_assert(SPLIT_FUSE_MAX_SIGS <= VERIFY_SPLIT_MAX_SIGS, "a fused launch must take the split kernel");

// k + sum_{p < comb_pos(W)} 2^(W-1) 2^(W p) for k < 2^253 (< 2^(W comb_pos(W)) for every window).
template <int W>
NW_HD void offset_scalar(uint32_t kp[9], const uint32_t k[8]) {
    uint64_t c = 0;
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        uint32_t add = 0;
#pragma unroll
        for (int p = 0; p < comb_pos(W); ++p) {
            const int bit = W * p + W - 1;
            if ((bit >> 5) == w) add |= 1u << (bit & 31);
        }
        c += (uint64_t)(w < 8 ? k[w] : 0u) + add;
        kp[w] = (uint32_t)c;
        c >>= 32;
    }
}

template <int W>
NW_HD void shift_window(uint32_t kp[9]) {
#pragma unroll
    for (int w = 0; w < 8; ++w) kp[w] = (kp[w] >> W) | (kp[w + 1] << (32 - W));
    kp[8] >>= W;
}

template <int W>
NW_HD int low_digit(const uint32_t kp[9]) {
    return (int)(kp[0] & ((1u << W) - 1u)) - (1 << (W - 1));
}

// FUSE (split_fuses_finish: launches of up to SPLIT_FUSE_MAX_SIGS signatures, one per k_finish lane):
// after the butterfly every lane of a group holds P, so all 8 lanes run k_finish's work for their
// signature (the inversion on a dense EXEC mask) and the group's first lane writes the verdict:
// no k_finish launch and no P round trip through pbuf (a single header / vote check: ~5 us).
template <int MSGMODE, int WA, bool FUSE>
__global__ void __launch_bounds__(256) k_verify_split(VerifyParams a) {
    constexpr int WB = B_WINDOW;
    constexpr int PB = comb_pos(WB), NPOS = PB + comb_pos(WA);
    constexpr int K = (NPOS + VERIFY_SPLIT - 1) / VERIFY_SPLIT;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t j = t % VERIFY_SPLIT;
    // whole signature groups exit together (VERIFY_SPLIT divides 64): the shuffles below see
    // only active partners.  A launch of fewer signatures than one wave holds (a lone header or
    // vote) runs duplicate groups on the rest of wave 0 (no writes): a wave with a sparse EXEC mask
    // issues its chain 1.2-1.4x slower.
    const uint32_t s_raw = t / VERIFY_SPLIT;
    // FUSE: a wave with any signature keeps all its lanes (duplicates past the launch's last group)
    // for the wave-batched inversion, which needs every lane of the wave
    if (s_raw >= a.gn && (FUSE ? (t & ~63u) >= a.gn * VERIFY_SPLIT : (a.gn * VERIFY_SPLIT >= 64 || t >= 64))) return;
    const bool owner = s_raw < a.gn;
    const uint32_t gid = a.g0 + (owner ? s_raw : s_raw % a.gn);
    const uint32_t i = a.perm ? a.perm[gid] : gid;
    uint32_t R[8], S[8], h[8], slot, kinfo, cert;
    const bool nocert = lane_inputs<MSGMODE>(a, i, R, S, slot, kinfo, cert, h);
    const bool sok = sc_is_canonical(S);
    const bool aok = (kinfo & KI_OK) != 0;
    uint32_t flags = (sok ? NW_F_S_OK : 0u) | (aok ? NW_F_A_OK : 0u) | ((kinfo & KI_SMALL) ? NW_F_A_SMALL : 0u) |
                     (nocert ? PF_NOCERT : 0u);
    const uint32_t tk = (kinfo >> KI_TORSION_SHIFT) & 7u;
    if (a.batch_mode && tk != 0 && sok && aok) {
        uint32_t z4[4];
        coeff_z(a, i, cert, z4);
        flags |= torsion_coef(z4, h, tk) << NW_F_TCOEF_SHIFT;
    }
    uint32_t sw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sw[k] = sok ? S[k] : 0u;
    uint32_t sp[9], hp[9];
    offset_scalar<WB>(sp, sw);
    offset_scalar<WA>(hp, h);
    // advance both recoders to this lane's first position (lane-dependent, cheap shifts)
    const int p0 = (int)j * K;
    for (int q = 0; q < p0 && q < PB; ++q) shift_window<WB>(sp);
    for (int q = PB; q < p0; ++q) shift_window<WA>(hp);
    const uint32_t* atab = a.key_tab + (size_t)slot * a.key_stride;
    // all K digits first (cheap shifts), so each table entry's 128-B gather can be issued one
    // position ahead, under the previous mixed addition (the entries are cold in L2: a lone
    // signature's chain would otherwise wait a full memory round trip per position)
    int dig[K];
#pragma unroll
    for (int st = 0; st < K; ++st) {
        const bool base = p0 + st < PB;
        dig[st] = base ? low_digit<WB>(sp) : low_digit<WA>(hp);
        if (base) shift_window<WB>(sp);
        else shift_window<WA>(hp);
    }
    auto negs = [&](int st) -> bool {
        const int pos = p0 + st;
        return pos < NPOS && (pos < PB ? dig[st] < 0 : dig[st] > 0);
    };
    // entries loaded in the order their digit's sign needs (load_ent_sw)
    auto entry = [&](int st) -> ent_sw {
        const int pos = p0 + st;
        const uint32_t ad = (uint32_t)(dig[st] < 0 ? -dig[st] : dig[st]);
        // past the last position: entry 0 of base position 0 (the identity), a no-op addition
        const uint32_t* e = pos >= NPOS ? a.btab
                            : pos < PB  ? a.btab + ((size_t)pos * comb_ent(WB) + ad) * PRECOMP_WORDS
                                        : atab + ((size_t)(pos - PB) * comb_ent(WA) + ad) * PRECOMP_WORDS;
        return load_ent_sw(e, negs(st));
    };
    ent_sw nx = entry(0);
    ge_p3 P;
#pragma unroll
    for (int st = 0; st < K; ++st) {
        const ent_sw cur = nx;
        if (st + 1 < K) nx = entry(st + 1);
        if (st == 0) P = ent_sw_first(cur, negs(st));
        else P = ge_madd_sgn(P, ent_sw_precomp(cur), lane_mask(negs(st)));
    }
#pragma unroll
    for (int off = 1; off < VERIFY_SPLIT; off <<= 1) {
        ge_p3 o;
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            o.X.v[k] = __shfl_xor(P.X.v[k], off, 64);
            o.Y.v[k] = __shfl_xor(P.Y.v[k], off, 64);
            o.Z.v[k] = __shfl_xor(P.Z.v[k], off, 64);
            o.T.v[k] = __shfl_xor(P.T.v[k], off, 64);
        }
        P = ge_add(P, ge_to_cached(o));
    }
    if constexpr (FUSE) {
        const bool emits = j == 0 && owner;   // the group's writer (the other lanes: same chain, no stores)
        uint32_t pf = verify_pflags(P, R, flags);
        if (emits) pf = park_mismatch(a, i, P, pf);
        // the wave's 8 signature groups share ONE inversion, on the scalar unit (nw_inv.h)
        const fe zi = fe_invert_batched<VERIFY_SPLIT>(P.Z);
        const uint32_t f = finish_x_flags(P.X, zi, pf);
        if (emits) finish_emit(a, i, pf, f);
        return;
    }
    if (j != 0 || !owner) return;
    store_prec_soa(a.pbuf, a.n, gid, P, park_mismatch(a, i, P, verify_pflags(P, R, flags)));
}

template <int WA>
hipError_t launch_split_wa(const VerifyParams& p, int msgmode, hipStream_t st) {
    const dim3 b(256), g(blocks_for((uint64_t)p.gn * VERIFY_SPLIT, 256));
    const bool fuse = split_fuses_finish(p.gn, p.fk);
    if (msgmode == 0) {
        if (fuse) hipLaunchKernelGGL((k_verify_split<0, WA, true>), g, b, 0, st, p);
        else hipLaunchKernelGGL((k_verify_split<0, WA, false>), g, b, 0, st, p);
    } else {
        if (fuse) hipLaunchKernelGGL((k_verify_split<1, WA, true>), g, b, 0, st, p);
        else hipLaunchKernelGGL((k_verify_split<1, WA, false>), g, b, 0, st, p);
    }
    return hipGetLastError();
}

}  // namespace nw
