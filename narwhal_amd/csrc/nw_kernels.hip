// gfx950 kernels for the Ed25519 verify + SHA-512 hot path.
//
// Verification strategy: for signature i with committee key A_i,
//     P_i = s_i B - h_i A_i          (two fixed-base combs, 32 mixed additions, no doublings)
// is compared with the signature's R encoding.  P_i == decode(R_i) is exactly dalek's strict
// equation (verify_strict).  The cofactorless batch equation of dalek::verify_batch with
// coefficients z_i,
//     sum_i [ z_i R_i + (z_i h_i mod l) A_i ] - (sum_i z_i s_i mod l) B == O,
// decomposes exactly (with D_i = R_i - P_i, A_i^t the 8-torsion part of A_i, l = 5 mod 8) into
//     sum_i z_i D_i  +  sum_i ((r_i - z_i h_i) mod 8) A_i^t == O,      r_i = z_i h_i mod l,
// so a certificate whose signatures all satisfy D_i = O and whose keys are torsion-free is accepted
// without any variable-base work; everything else goes to the exact path (k_slow_prep, k_slow_mul),
// which decides the remaining terms exactly.  Verdicts are therefore identical to dalek's for every
// input (not just honest ones) given the same z_i.
//
// Pipeline per batch: k_prep_certs + k_expand_count -> [signer grouping] -> k_verify (P_i, one lane per signature)
// -> k_finish (Montgomery batch inversion of Z over FINISH_K signatures per lane, encoding match,
// strict verdict) -> k_slow_prep / k_slow_mul (compacted list of mismatches only) -> k_cert_finalize.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include "nw_point.h"
#include "nw_sha512.h"
#include "nw_kernels.h"
#include "nw_core.h"
#include "nw_quad.h"

namespace nw {

template <int WA>
hipError_t launch_vs_wa(const VerifyParams& p, int msgmode, bool slow, uint32_t n_upper, hipStream_t st);
extern template hipError_t launch_vs_wa<8>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<9>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<12>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<13>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<16>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<20>(const VerifyParams&, int, bool, uint32_t, hipStream_t);

// ------------------------------------------------------------------------------------ signer grouping
// Counting sort of signature indices by key-cache slot: perm lists the signatures of slot 0, then
// slot 1, ...  (order inside a slot is arbitrary; every output is written at the original index).
// Committees are small next to a batch (100 keys, 1M signatures), so global per-slot atomics would
// serialize: each workgroup histograms a GROUP_TILE-signature tile in LDS and touches global
// memory once per (tile, slot).  Above GROUP_LDS_KEYS slots the plain global-atomic form is used
// (contention is then spread over many addresses anyway).
static constexpr uint32_t GROUP_TILE = 4096;
static constexpr uint32_t GROUP_LDS_KEYS = 8192;

// Out-of-range slots (rejected by k_verify) are grouped with slot 0 so no access leaves the arrays.
__device__ __forceinline__ uint32_t clamp_slot(uint32_t s, uint32_t nkeys) { return s < nkeys ? s : 0u; }

// Single-block exclusive scan of counts[0..k) into cursor[0..k).
__global__ void __launch_bounds__(1024) k_scan_slots(uint32_t k, const uint32_t* counts, uint32_t* cursor) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (k + 1023) / 1024;
    const uint32_t b = t * per, e = min(k, b + per);
    uint32_t sum = 0;
    for (uint32_t j = b; j < e; ++j) sum += counts[j];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;   // exclusive prefix of this thread's chunk
    for (uint32_t j = b; j < e; ++j) {
        const uint32_t c = counts[j];
        cursor[j] = run;
        run += c;
    }
}

__global__ void __launch_bounds__(256) k_scatter_slots(uint32_t n, uint32_t nkeys, const uint32_t* signer,
                                                       uint32_t* cursor, uint32_t* perm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) perm[atomicAdd(&cursor[clamp_slot(signer[i], nkeys)], 1u)] = i;
}

// Tile-local scatter: LDS histogram -> one global atomic per (tile, slot) reserves the tile's run
// of each slot -> LDS atomics rank the tile's signatures inside their runs.
__global__ void __launch_bounds__(256) k_scatter_slots_lds(uint32_t n, uint32_t nkeys, const uint32_t* signer,
                                                           uint32_t* cursor, uint32_t* perm) {
    extern __shared__ uint32_t lds[];
    uint32_t* base = lds;            // [nkeys] tile count, then the tile's global base
    uint32_t* rank = lds + nkeys;    // [nkeys] running rank inside the tile
    for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x) {
        base[k] = 0;
        rank[k] = 0;
    }
    __syncthreads();
    const uint32_t t0 = blockIdx.x * GROUP_TILE;
    const uint32_t t1 = min(n, t0 + GROUP_TILE);
    for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) atomicAdd(&base[clamp_slot(signer[i], nkeys)], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x)
        if (base[k]) base[k] = atomicAdd(&cursor[k], base[k]);
    __syncthreads();
    for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
        const uint32_t k = clamp_slot(signer[i], nkeys);
        perm[base[k] + atomicAdd(&rank[k], 1u)] = i;
    }
}

// ------------------------------------------------------------------------------------ finish
// Montgomery batch inversion of the Z of FINISH_K signatures per lane (one field inversion per
// chunk), affine x, y, encoding match against R, strict verdict, and (batch mode) compaction of the
// mismatching signatures into the exact-path list.  Lane L of NL owns the processing-order columns
// g = L, L + NL, L + 2 NL, ... so every pbuf / pre access of a wave is one contiguous 256-B run.
// ONE (a.fk == 1: finish_k_for gives it to launches of up to 256 x 4 x 64 = 262,144 signatures,
// i.e. every latency-bound call and mid-size batches up to one lane per SIMD slot): its own kernel,
// so the chunked path's register allocation is untouched.
template <bool ONE>
__global__ void __launch_bounds__(256) k_finish(VerifyParams a) {
    const uint32_t NL = (a.gn + a.fk - 1) / a.fk;
    const uint32_t Lr = blockIdx.x * blockDim.x + threadIdx.x;
    // fewer lanes than a wave (one header or vote signature: ONE inversion on one lane): the idle
    // lanes of wave 0 run duplicates (no writes), since a wave with a sparse EXEC mask issues its
    // chain 1.2-1.4x slower
    if (Lr >= NL && (NL >= 64 || Lr >= 64)) return;
    const bool owner = Lr < NL;
    const uint32_t L = owner ? Lr : Lr % NL;
    const uint32_t cnt = (a.gn - L + NL - 1) / NL;   // columns g0 + L + k NL < g0 + gn  (cnt <= fk)
    const size_t n = a.n;
    const size_t gbase = (size_t)a.g0 + L;
    auto emit = [&](uint32_t i, uint32_t pf, uint32_t f) { finish_emit(a, i, pf, f); };
    if constexpr (ONE) {
        // one signature per lane: every load issued before the inversion, no prefix products
        const fe z = load_fe_soa(a.pbuf + 10 * n, n, gbase);
        const fe X = load_fe_soa(a.pbuf, n, gbase);
        const uint32_t pf = a.pbuf[PREC_FLAGS_ROW * n + gbase];
        const uint32_t i = a.perm ? a.perm[gbase] : (uint32_t)gbase;
        const fe zi = (NW_INV_VAR && a.gn <= 8) ? fe_invert_var(z) : fe_invert_sg(z);
        const uint32_t f = finish_x_flags(X, zi, pf);
        if (owner) emit(i, pf, f);
        return;
    } else {
        // Both chains are fully unrolled over FINISH_K (guarded by cnt) so the column loads are
        // independent of the running products and issue ahead of them: with one wave per SIMD the
        // kernel is latency-bound, and a load inside the serial chain would stall it every step.
        const uint32_t* zrow = a.pbuf + 10 * n;
        fe acc = fe_one();
#pragma unroll
        for (int k = 0; k < FINISH_K; ++k) {
            if ((uint32_t)k < cnt) {
                const size_t g = gbase + (size_t)k * NL;
                acc = fe_mul(acc, load_fe_soa(zrow, n, g));
                store_fe_soa(a.pre, n, g, acc);   // duplicates store the owner's own values (scratch)
            }
        }
        // Inversion: variable-time safegcd (public data) when each lane chains several signatures
        // (throughput-bound launches: fewer instructions on average); the branch-free constant-time
        // divsteps for one signature per lane (latency-bound launches: with 64 independent inversions
        // per wave the variable-time loop runs the slowest lane's count, measured 10% slower there:
        // profiles/r02/ab_r02.txt).  a.fk is uniform, so the branch does not diverge.
        // A launch of a handful of signatures (one header / vote signature) has a handful of active
        // lanes, so the variable-time loop's cost is that one lane's own count: variable time again.
        fe inv;
        if (NW_INV_VAR && (a.fk >= 4 || a.gn <= 8)) inv = fe_invert_var(acc);
        else inv = fe_invert_sg(acc);
#pragma unroll
        for (int k = FINISH_K - 1; k >= 0; --k) {
            if ((uint32_t)k < cnt) {
                const size_t g = gbase + (size_t)k * NL;
                fe zi = inv;
                if (k > 0) {
                    zi = fe_mul(inv, load_fe_soa(a.pre, n, g - NL));
                    inv = fe_mul(inv, load_fe_soa(zrow, n, g));
                }
                const uint32_t i = a.perm ? a.perm[g] : (uint32_t)g;
                const uint32_t pf = a.pbuf[PREC_FLAGS_ROW * n + g];
                const uint32_t f = finish_x_flags(load_fe_soa(a.pbuf, n, g), zi, pf);
                if (owner) emit(i, pf, f);
            }
        }
    }
}

// Per-certificate verdict: definitive Err on any bad S / undecodable A / undecodable R, else the
// exact remaining batch sum (usually empty) must be the identity.  One 64-lane wave per
// certificate: lanes stride over the votes (coalesced flag reads), wave reductions combine them;
// the exact sum over slow-path terms (failing certificates only) is a lane-strided sum + shuffle tree.
// One wave per certificate: flag reduction, stake sum, and the verdict whenever the flags decide it
// (parse / decode failure, all votes matching, one term with a prime-order component).  The rest
// (two or more slow-path terms) is appended to the exact list for k_cert_exact, which has the
// registers for the point sum: this kernel stays at a handful of VGPRs and never spills.
// Certificate c's finalize, by one wave (lane = 0..63).
__device__ __forceinline__ void finalize_cert(const FinalizeParams& a, uint32_t c, uint32_t lane) {
    const uint32_t first = a.cert_first[c];
    // a vote range past the signature array (device inputs are not host-checked) rejects the
    // certificate; only the in-range votes are read
    const bool range_bad = (uint64_t)first + a.cert_n[c] > a.nsigs;
    const uint32_t nv = range_bad ? (first < a.nsigs ? a.nsigs - first : 0u) : a.cert_n[c];
    // CS_DOOM: a bad S / undecodable A (the flags say so too) or a vote range overlapping another
    // certificate's (k_expand_count)
    bool bad = range_bad || (a.cert_state && (a.cert_state[c] & CS_DOOM)), slow = false;
    uint32_t tsum = 0;
    uint64_t stake = 0;
    for (uint32_t v = lane; v < nv; v += 64) {
        const uint32_t f = a.flags[first + v];
        // a vote this certificate does not own (overlapping device ranges, NW_ERR_ARG) was checked
        // against its owner's message: it rejects this certificate and adds none of its stake
        const bool own = a.sig_cert[first + v] == c;
        bad = bad || !own || ((f & (NW_F_S_OK | NW_F_A_OK)) != (NW_F_S_OK | NW_F_A_OK)) || (f & NW_F_R_BAD);
        slow = slow || (f & NW_F_SLOW);
        tsum += (f >> NW_F_TCOEF_SHIFT) & 7u;
        if (own && (f & NW_F_STRICT)) stake += a.stake[a.signer[first + v]];
    }
    bad = __any(bad);
    slow = __any(slow);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        tsum += __shfl_xor(tsum, off, 64);
        stake += __shfl_xor(stake, off, 64);
    }
    if (lane != 0) return;
    if (a.accepted_stake) a.accepted_stake[c] = stake;
    bool ok;
    if (bad) {
        ok = false;
    } else if (!slow) {
        ok = (tsum & 7u) == 0;
    } else if ((a.cert_state[c] & CS_BIG_MASK) == 1u) {
        ok = false;   // one term with a prime-order component: the sum cannot be the identity (k_slow_prep)
    } else {
        a.exact_list[atomicAdd(a.exact_count, 1u)] = c;   // the exact sum writes the verdict
        return;
    }
    if (a.cert_ok) a.cert_ok[c] = ok ? 1 : 0;
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
    __syncthreads();
    acc = lane < k ? load_p3(part[lane]) : ge_identity();
    __syncthreads();   // part is rewritten by the next listed certificate
    for (uint32_t off = 1; off < k; off <<= 1) {   // k is wave-uniform
        const ge_p3 o = ge_shfl_down(acc, off);
        acc = ge_select(acc, ge_add(acc, ge_to_cached(o)), lane + off < k);
    }
    if (lane == 0 && a.cert_ok) a.cert_ok[c] = (!bad && ge_is_identity(acc)) ? 1 : 0;
}

// Per-certificate verdict: definitive Err on any bad S / undecodable A / undecodable R, else the
// exact remaining batch sum (usually empty) must be the identity.  One wave per certificate: flag
// reduction, stake sum, and the verdict whenever the flags decide it (parse / decode failure, all
// votes matching, one term with a prime-order component).  The rest (two or more slow-path terms)
// is appended to the exact list for k_cert_exact, which has the registers for the point sum: this
// kernel stays at a handful of VGPRs and never spills.
__global__ void __launch_bounds__(256) k_cert_finalize(FinalizeParams a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (a.sig_ok) {   // strict verdict bytes of every signature (the flags are final here)
        const uint32_t nthr = gridDim.x * blockDim.x;
        for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < a.nsigs; v += nthr)
            a.sig_ok[v] = (a.flags[v] & NW_F_STRICT) ? 1 : 0;
    }
    if (c >= a.ncerts) return;   // whole wave exits together
    finalize_cert(a, c, lane);
}

static constexpr uint32_t EXACT_MAX_BLOCKS = 1024;
__global__ void __launch_bounds__(64) k_cert_exact(FinalizeParams a) {
    __shared__ uint32_t part[64][40];
    const uint32_t cnt = *a.exact_count;
    for (uint32_t e = blockIdx.x; e < cnt; e += gridDim.x) exact_cert(a, a.exact_list[e], threadIdx.x, part);
}

// Both in one wave for calls of a few certificates (a single certificate, header batch or vote
// batch): one launch instead of two (~5 us each even when the exact list is empty).  The wave reads
// back the exact list its own lanes appended: a device-scope fence and atomic reads order them.
static constexpr uint32_t TAIL_MAX_CERTS = 16;
__global__ void __launch_bounds__(64) k_cert_tail(FinalizeParams a) {
    __shared__ uint32_t part[64][40];
    const uint32_t lane = threadIdx.x;
    if (a.sig_ok)
        for (uint32_t v = lane; v < a.nsigs; v += 64) a.sig_ok[v] = (a.flags[v] & NW_F_STRICT) ? 1 : 0;
    for (uint32_t c = 0; c < a.ncerts; ++c) finalize_cert(a, c, lane);
    __threadfence();
    __syncthreads();
    const uint32_t cnt = __hip_atomic_load(a.exact_count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t e = 0; e < cnt; ++e)
        exact_cert(a, __hip_atomic_load(a.exact_list + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), lane, part);
}

// ------------------------------------------------------------------------------------ batch preamble
// Two launches replace the five small ones a certificate batch used to start with (status /
// sig_cert / slot-count fills, input check, certificate expansion, slot histogram): ~5 us each on
// MI355X, dominated by dispatch, not work.
//   k_prep_certs:   sig_cert = NO_CERT (a vote outside every certificate gets no verdict and no
//                   exact-path entry), the slot counts, the slow-path counter and the status word = 0.
//   k_expand_count: block b expands certificates [4 b, 4 b + 4) into sig_cert (a vote already
//                   claimed by another certificate is NW_ERR_ARG: ranges must be disjoint) and, for
//                   signature tile b (GROUP_TILE signatures), histograms the signer slots (LDS, one
//                   global add per slot) and/or checks them; every check ORs NW_ERR_ARG into status.
//   Device inputs are checked here and nowhere else: vote ranges inside [0, nsigs), pairwise
//   disjoint, signer slots inside the key cache.
__global__ void __launch_bounds__(256) k_prep_certs(uint32_t nsigs, uint32_t nkeys, uint32_t* sig_cert, uint32_t* counts,
                                                    uint32_t* zero4, uint32_t* status, uint32_t ncerts,
                                                    uint32_t* cert_state) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = t; i <= nsigs; i += stride) sig_cert[i] = NO_CERT;
    if (cert_state)
        for (uint32_t c = t; c < ncerts; c += stride) cert_state[c] = 0u;
    if (counts)
        for (uint32_t k = t; k < nkeys; k += stride) counts[k] = 0u;
    if (t < 4) zero4[t] = 0u;
    if (status && t == 0) *status = 0u;
}

static constexpr uint32_t EXPAND_CERTS_PER_BLOCK = 4;   // one wave each
__global__ void __launch_bounds__(256) k_expand_count(uint32_t ncerts, uint32_t nsigs, uint32_t nkeys,
                                                      const uint32_t* cert_first, const uint32_t* cert_n,
                                                      const uint32_t* signer, uint32_t* sig_cert, uint32_t* counts,
                                                      uint32_t* status, uint32_t* cert_state) {
    extern __shared__ uint32_t hist[];
    // one wave per certificate: its lanes write the vote -> certificate entries side by side (a
    // thread per certificate would store 667 / 6,667 entries serially at C3 / C4)
    const uint32_t c = blockIdx.x * EXPAND_CERTS_PER_BLOCK + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    bool bad = false;
    if (c < ncerts) {
        const uint32_t f = cert_first[c], n = cert_n[c];
        bad = lane == 0 && (uint64_t)f + n > nsigs;
        const uint32_t end = (uint64_t)f + n > nsigs ? nsigs : f + n;   // clamped: k_cert_finalize rejects it
        for (uint32_t v = f + lane; v < end; v += 64) {
            const uint32_t prev = atomicExch(&sig_cert[v], c);
            if (prev != NO_CERT) {
                // a vote claimed twice: whichever certificate the map ends with checks it against its
                // own message, so BOTH are doomed (k_cert_finalize rejects them), in any order
                bad = true;
                if (cert_state) {
                    atomicOr(&cert_state[c], CS_DOOM);
                    if (prev < ncerts) atomicOr(&cert_state[prev], CS_DOOM);
                }
            }
        }
    }
    const uint32_t t0 = blockIdx.x * GROUP_TILE;
    if ((counts || status) && t0 < nsigs) {
        const uint32_t t1 = min(nsigs, t0 + GROUP_TILE);
        const bool lds = counts && nkeys <= GROUP_LDS_KEYS;
        if (lds) {
            for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x) hist[k] = 0;
            __syncthreads();
        }
        for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
            const uint32_t sl = signer[i];
            bad = bad || sl >= nkeys;
            if (lds)
                atomicAdd(&hist[clamp_slot(sl, nkeys)], 1u);
            else if (counts)
                atomicAdd(&counts[clamp_slot(sl, nkeys)], 1u);
        }
        if (lds) {
            __syncthreads();
            for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x)
                if (hist[k]) atomicAdd(&counts[k], hist[k]);
        }
    }
    if (bad && status) atomicOr(status, (uint32_t)NW_ERR_ARG);
}

__global__ void __launch_bounds__(256) k_flags_to_ok(uint32_t n, const uint32_t* flags, uint8_t* ok) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ok[i] = (flags[i] & NW_F_STRICT) ? 1 : 0;
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
__global__ void __launch_bounds__(256) k_slow_mul(VerifyParams a) {
    __shared__ uint32_t tab[SLOW_MUL_QUADS][8][40];
    const uint32_t cnt = *a.slow_count;
    const uint32_t qd = threadIdx.x >> 2, q = threadIdx.x & 3u;
    uint32_t (*T)[40] = tab[qd];
    // entries dealt to the blocks first (one wave each), as in k_slow_prep: a wave's time is one
    // chain whatever its number of quads, so spreading the entries keeps the waves short and apart.
    // A wave with fewer entries than quads runs duplicate chains of its own entries on the idle
    // quads (own LDS table slot, no record writes), so its EXEC mask stays full.
    const uint32_t wq = (threadIdx.x & 63u) >> 2;                    // quad index inside the wave
    for (uint32_t base = (qd - wq) * gridDim.x + blockIdx.x; base < cnt; base += gridDim.x * SLOW_MUL_QUADS) {
        const uint32_t t_own = base + wq * gridDim.x;
        const uint32_t v = (uint32_t)__popcll(__ballot(t_own < cnt)) >> 2;   // entries of this wave: quads [0, v)
        const bool owner = wq < v;
        const uint32_t t = owner ? t_own : base + (wq % v) * gridDim.x;
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

// ------------------------------------------------------------------------------------ launchers
static hipError_t launch_vs(const VerifyParams& p, int msgmode, int key_window, bool slow, uint32_t n_upper,
                            hipStream_t st) {
    switch (key_window) {
        case 8: return launch_vs_wa<8>(p, msgmode, slow, n_upper, st);
        case 9: return launch_vs_wa<9>(p, msgmode, slow, n_upper, st);
        case 12: return launch_vs_wa<12>(p, msgmode, slow, n_upper, st);
        case 13: return launch_vs_wa<13>(p, msgmode, slow, n_upper, st);
        case 16: return launch_vs_wa<16>(p, msgmode, slow, n_upper, st);
        case 20: return launch_vs_wa<20>(p, msgmode, slow, n_upper, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_verify(const VerifyParams& p, int msgmode, int key_window, hipStream_t st) {
    if (p.gn == 0) return hipSuccess;
    return launch_vs(p, msgmode, key_window, false, 0, st);
}

hipError_t launch_slow(const VerifyParams& p, int msgmode, int key_window, uint32_t n_upper, hipStream_t st) {
    if (n_upper == 0) return hipSuccess;
    hipError_t e = launch_vs(p, msgmode, key_window, true, n_upper, st);
    if (e != hipSuccess) return e;
    const uint32_t nb = std::min<uint32_t>(blocks_for(n_upper, SLOW_MUL_QUADS), 256u);
    hipLaunchKernelGGL(k_slow_mul, dim3(nb), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_finish(const VerifyParams& p, hipStream_t st) {
    if (p.gn == 0) return hipSuccess;
    if (p.fk < 1 || p.fk > (uint32_t)FINISH_K || (uint64_t)p.g0 + p.gn > p.n) return hipErrorInvalidValue;
    const uint64_t lanes = (p.gn + p.fk - 1) / p.fk;
    if (p.fk == 1) hipLaunchKernelGGL(k_finish<true>, dim3(blocks_for(lanes, 256)), dim3(256), 0, st, p);
    else hipLaunchKernelGGL(k_finish<false>, dim3(blocks_for(lanes, 256)), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeParams& p, hipStream_t st) {
    if (p.ncerts == 0) return hipSuccess;
    if (p.ncerts <= TAIL_MAX_CERTS && p.nsigs <= 64u * 1024u) {
        hipLaunchKernelGGL(k_cert_tail, dim3(1), dim3(64), 0, st, p);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_cert_finalize, dim3(blocks_for((uint64_t)p.ncerts * 64, 256)), dim3(256), 0, st, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the exact list's length is on the device: a capped grid that exits at once when it is empty
    hipLaunchKernelGGL(k_cert_exact, dim3(std::min<uint32_t>(p.ncerts, EXACT_MAX_BLOCKS)), dim3(64), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_prep_expand(uint32_t ncerts, uint32_t nsigs, uint32_t nkeys, const uint32_t* first,
                              const uint32_t* nv, const uint32_t* signer, uint32_t* sig_cert, uint32_t* zero4,
                              uint32_t* counts, uint32_t* status, uint32_t* cert_state, hipStream_t st) {
    const uint32_t prep_blocks = std::min<uint32_t>(blocks_for(std::max(nsigs + 1, ncerts), 256), 1024u);
    hipLaunchKernelGGL(k_prep_certs, dim3(prep_blocks), dim3(256), 0, st, nsigs, nkeys, sig_cert, counts, zero4, status,
                       ncerts, cert_state);
    const bool tiles = (counts || status) && nsigs > 0;
    const uint32_t nb = std::max<uint32_t>(blocks_for(ncerts, EXPAND_CERTS_PER_BLOCK), tiles ? blocks_for(nsigs, GROUP_TILE) : 0u);
    if (nb == 0) return hipGetLastError();
    const size_t lds = counts && nkeys <= GROUP_LDS_KEYS ? (size_t)nkeys * 4 : 0;
    hipLaunchKernelGGL(k_expand_count, dim3(nb), dim3(256), lds, st, ncerts, nsigs, nkeys, first, nv, signer, sig_cert,
                       counts, status, cert_state);
    return hipGetLastError();
}

// Scan + scatter of the signer grouping whose counts k_expand_count produced.
hipError_t launch_group_scatter(uint32_t n, uint32_t nkeys, const uint32_t* signer, const uint32_t* counts,
                                uint32_t* cursor, uint32_t* perm, hipStream_t st) {
    if (n == 0 || nkeys == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_slots, dim3(1), dim3(1024), 0, st, nkeys, counts, cursor);
    if (nkeys <= GROUP_LDS_KEYS)
        hipLaunchKernelGGL(k_scatter_slots_lds, dim3(blocks_for(n, GROUP_TILE)), dim3(256), nkeys * 8, st, n, nkeys,
                           signer, cursor, perm);
    else
        hipLaunchKernelGGL(k_scatter_slots, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, nkeys, signer, cursor,
                           perm);
    return hipGetLastError();
}

hipError_t launch_flags_to_ok(uint32_t n, const uint32_t* flags, uint8_t* ok, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_flags_to_ok, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, flags, ok);
    return hipGetLastError();
}

}  // namespace nw
