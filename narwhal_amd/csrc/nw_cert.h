// Certificate verdicts of the batch equation, by one wave per certificate: the finalize (flag
// reduction, stake sum, verdict whenever the flags decide it) and the exact sum over slow-path
// terms.  LDS exchanges between the wave's lanes use wave_lds_sync (nw_core.h): a caller may run a
// certificate on one wave of a workgroup whose other waves have finished.  Shared by k_cert_finalize / k_cert_exact / k_cert_tail (nw_kernels.hip) and by the
// small-call exact-path kernel k_slow_tail (nw_verify_kernels.h).
#pragma once
#include <hip/hip_runtime.h>
#include "nw_point.h"
#include "nw_kernels.h"
#include "nw_core.h"

namespace nw {

// Per-certificate verdict: definitive Err on any bad S / undecodable A / undecodable R, else the
// exact remaining batch sum (usually empty) must be the identity.  The flag reduction, stake sum,
// and the verdict whenever the flags decide it (parse / decode failure, all votes matching, one
// term with a prime-order component) are the finalize; the rest (two or more slow-path terms) is
// appended to the exact list for k_cert_exact, which has the registers for the point sum: the
// finalize stays at a handful of VGPRs and never spills.  A certificate's votes are scanned by one
// wave (finalize_cert) or, for large certificates, by a whole workgroup (k_cert_finalize_wg:
// C4's 6,667 votes are 105 dependent load rounds for one wave, 7 for sixteen).
struct FinalizeAcc {
    bool bad, slow;
    uint32_t tsum;
    uint64_t stake;
};

// The votes t, t + stride, ... of certificate c (lanes stride over them: coalesced flag reads),
// reduced over the calling wave: every lane returns the wave's totals.
__device__ __forceinline__ FinalizeAcc finalize_scan(const FinalizeParams& a, uint32_t c, uint32_t t, uint32_t stride) {
    const uint32_t first = a.cert_first[c];
    // a vote range past the signature array (device inputs are not host-checked) rejects the
    // certificate; only the in-range votes are read
    const bool range_bad = (uint64_t)first + a.cert_n[c] > a.nsigs;
    const uint32_t nv = range_bad ? (first < a.nsigs ? a.nsigs - first : 0u) : a.cert_n[c];
    // CS_DOOM: a bad S / undecodable A (the flags say so too) or a vote range overlapping another
    // certificate's (k_expand_count)
    FinalizeAcc r{range_bad || (a.cert_state && (a.cert_state[c] & CS_DOOM)), false, 0u, 0u};
    for (uint32_t v = t; v < nv; v += stride) {
        const uint32_t f = a.flags[first + v];
        // a vote this certificate does not own (overlapping device ranges, NW_ERR_ARG) was checked
        // against its owner's message: it rejects this certificate and adds none of its stake
        const bool own = a.sig_cert[first + v] == c;
        r.bad = r.bad || !own || ((f & (NW_F_S_OK | NW_F_A_OK)) != (NW_F_S_OK | NW_F_A_OK)) || (f & NW_F_R_BAD);
        r.slow = r.slow || (f & NW_F_SLOW);
        r.tsum += (f >> NW_F_TCOEF_SHIFT) & 7u;
        if (own && (f & NW_F_STRICT)) r.stake += a.stake[a.signer[first + v]];
    }
    r.bad = __any(r.bad);
    r.slow = __any(r.slow);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        r.tsum += __shfl_xor(r.tsum, off, 64);
        r.stake += __shfl_xor(r.stake, off, 64);
    }
    return r;
}

// Certificate c's verdict from its totals (one thread).
__device__ __forceinline__ void finalize_decide(const FinalizeParams& a, uint32_t c, const FinalizeAcc& r) {
    if (a.accepted_stake) a.accepted_stake[c] = r.stake;
    bool ok;
    if (r.bad) {
        ok = false;
    } else if (!r.slow) {
        ok = (r.tsum & 7u) == 0;
    } else if ((a.cert_state[c] & CS_BIG_MASK) == 1u) {
        ok = false;   // one term with a prime-order component: the sum cannot be the identity (k_slow_prep)
    } else {
        a.exact_list[atomicAdd(a.exact_count, 1u)] = c;   // the exact sum writes the verdict
        return;
    }
    if (a.cert_ok) a.cert_ok[c] = ok ? 1 : 0;
}

// Certificate c's finalize, by one wave (lane = 0..63).
__device__ __forceinline__ void finalize_cert(const FinalizeParams& a, uint32_t c, uint32_t lane) {
    const FinalizeAcc r = finalize_scan(a, c, lane, 64);
    if (lane == 0) finalize_decide(a, c, r);
}

// Exact sum of listed certificate c, by one wave (lane = 0..63; part: the wave's LDS rows): every
// slow vote's record holds its term z_i D_i (k_slow_mul for prime-order components, k_slow_prep's
// (z_i mod 8) D_i for small-order ones), the torsion coefficients of the matching votes add
// (sum mod 8) T8.  Lanes sum their votes' terms, the lanes that hold a term are compacted through
// LDS, and a shuffle tree of ceil(log2(count)) levels adds them: the serial chain is a few point
// additions, not six levels plus per-term multiples.
__device__ __forceinline__ void exact_cert(const FinalizeParams& a, uint32_t c, uint32_t lane, uint32_t (*part)[40]) {
    const uint32_t first = a.cert_first[c], nv = a.cert_n[c];   // in range: bad ranges never get listed
    ge_p3 acc = ge_to_vgpr(ge_identity());
    bool has = false, bad = false;
    uint32_t tsum = 0;
    for (uint32_t v = lane; v < nv; v += 64) {
        const uint32_t f = a.flags[first + v];
        tsum += (f >> NW_F_TCOEF_SHIFT) & 7u;
        if (f & NW_F_SLOW) {
            const uint32_t* rec = a.slow_buf + (size_t)a.slow_slot[first + v] * SLOW_WORDS;
            // a term must be final and this certificate's own (valid calls always satisfy both;
            // a vote claimed by two certificates is NW_ERR_ARG and must not be accepted here)
            const uint32_t kind = rec[SLOW_KIND];
            if (a.sig_cert[first + v] != c || (kind != SK_SMALL && kind != SK_MUL)) {
                bad = true;
                continue;
            }
            const ge_p3 q = load_p3(rec);
            acc = has ? ge_add(acc, ge_to_cached(q)) : q;
            has = true;
        }
    }
    bad = __any(bad);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tsum += __shfl_xor(tsum, off, 64);
    const uint32_t tk = tsum & 7u;
    if (lane == 63 && tk != 0) {   // lane 63 adds (tk) T8 to its partial (binary: T8, 2 T8, 4 T8)
        const ge_p3 t1 = ge_t8(), t2 = ge_dbl(t1), t4 = ge_dbl(t2);
        ge_p3 t = ge_select(ge_identity(), t1, (tk & 1u) != 0);
        t = ge_add(t, ge_to_cached(ge_select(ge_identity(), t2, (tk & 2u) != 0)));
        t = ge_add(t, ge_to_cached(ge_select(ge_identity(), t4, (tk & 4u) != 0)));
        acc = has ? ge_add(acc, ge_to_cached(t)) : t;
        has = true;
    }
    const uint64_t mask = __ballot(has);
    const uint32_t k = (uint32_t)__popcll(mask);
    if (has) store_p3(part[__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))], acc);
    wave_lds_sync();
    acc = lane < k ? load_p3(part[lane]) : ge_identity();
    wave_lds_sync();   // part is rewritten by the next listed certificate
    for (uint32_t off = 1; off < k; off <<= 1) {   // k is wave-uniform
        const ge_p3 o = ge_shfl_down(acc, off);
        acc = ge_select(acc, ge_add(acc, ge_to_cached(o)), lane + off < k);
    }
    if (lane == 0 && a.cert_ok) a.cert_ok[c] = (!bad && ge_is_identity(acc)) ? 1 : 0;
}

// Calls of at most TAIL_MAX_CERTS certificates: the strict verdict bytes, every finalize, then the
// exact sums of the certificates the same wave listed, in one wave.
__device__ __forceinline__ void cert_tail(const FinalizeParams& a, uint32_t lane, uint32_t (*part)[40]) {
    if (a.sig_ok)
        for (uint32_t v = lane; v < a.nsigs; v += 64) a.sig_ok[v] = (a.flags[v] & NW_F_STRICT) ? 1 : 0;
    for (uint32_t c = 0; c < a.ncerts; ++c) finalize_cert(a, c, lane);
    __threadfence();
    __builtin_amdgcn_wave_barrier();
    const uint32_t cnt = __hip_atomic_load(a.exact_count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t e = 0; e < cnt; ++e)
        exact_cert(a, __hip_atomic_load(a.exact_list + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), lane, part);
}

}  // namespace nw
