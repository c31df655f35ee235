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
// Small calls (<= 16 certificates, <= 256 signatures) run everything after k_verify_split's fused finish
// as one workgroup: k_slow_tail (nw_verify_kernels.h).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include "nw_point.h"
#include "nw_sha512.h"
#include "nw_kernels.h"
#include "nw_core.h"
#include "nw_quad.h"
#include "nw_cert.h"
#include "nw_verify_kernels.h"

namespace nw {

template <int WA>
hipError_t launch_vs_wa(const VerifyParams& p, int msgmode, bool slow, uint32_t n_upper, hipStream_t st);
extern template hipError_t launch_vs_wa<8>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<9>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<12>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<13>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<16>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_vs_wa<20>(const VerifyParams&, int, bool, uint32_t, hipStream_t);
extern template hipError_t launch_slow_tail_wa<8>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);
extern template hipError_t launch_slow_tail_wa<9>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);
extern template hipError_t launch_slow_tail_wa<12>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);
extern template hipError_t launch_slow_tail_wa<13>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);
extern template hipError_t launch_slow_tail_wa<16>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);
extern template hipError_t launch_slow_tail_wa<20>(const VerifyParams&, const FinalizeParams&, int, hipStream_t);

// ------------------------------------------------------------------------------------ signer grouping
// Counting sort of signature indices by key-cache slot: perm lists the signatures of slot 0, then
// slot 1, ...  (order inside a slot is arbitrary; every output is written at the original index).
// Committees are small next to a batch (100 keys, 1M signatures), so global per-slot atomics would
// serialize: each workgroup histograms a GROUP_TILE-signature tile in LDS and touches global
// memory once per (tile, slot).  Above GROUP_LDS_KEYS slots the plain global-atomic form is used
// (contention is then spread over many addresses anyway).
#ifndef NW_GROUP_TILE
#define NW_GROUP_TILE 4096
#endif
static constexpr uint32_t GROUP_TILE = NW_GROUP_TILE;
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
                                                       const uint32_t* sig_cert, uint32_t* cursor, uint32_t* perm,
                                                       uint2* pinfo) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t s = signer[i];
        const uint32_t g = atomicAdd(&cursor[clamp_slot(s, nkeys)], 1u);
        perm[g] = i;
        pinfo[g] = make_uint2(s, sig_cert[i]);
    }
}

// Tile-local scatter: LDS histogram -> one global atomic per (tile, slot) reserves the tile's run
// of each slot -> LDS atomics rank the tile's signatures inside their runs.
__global__ void __launch_bounds__(256) k_scatter_slots_lds(uint32_t n, uint32_t nkeys, const uint32_t* signer,
                                                           const uint32_t* sig_cert, uint32_t* cursor, uint32_t* perm,
                                                           uint2* pinfo) {
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
        const uint32_t s = signer[i];
        const uint32_t g = base[clamp_slot(s, nkeys)] + atomicAdd(&rank[clamp_slot(s, nkeys)], 1u);
        perm[g] = i;
        pinfo[g] = make_uint2(s, sig_cert[i]);   // the raw slot: k_verify does its own range check
    }
}

// ------------------------------------------------------------------------------------ finish
// Montgomery batch inversion of the Z of up to FINISH_K signatures per lane, affine x, y, encoding
// match against R, strict verdict, and (batch mode) compaction of the mismatching signatures into
// the exact-path list.  Lane L of NL owns the processing-order columns g = L, L + NL, L + 2 NL, ...
// so every pbuf / pre access of a wave is one contiguous 256-B run.
// ONE (a.fk == 1: finish_k_for gives it to launches of up to 256 x 4 x 64 = 65,536 signatures, i.e.
// every latency-bound call, one wave per SIMD slot): no prefix products, one wave-batched inversion.
// Chunked (fk >= 2): the two chains are plain loops (124 VGPRs, four waves per SIMD, the next
// column's load issued one step ahead) and the workgroup's 256 lane products share ONE scalar-unit
// inversion (fe_invert_block).  Round 6 first ran the chains fully unrolled with every load hoisted
// (256 VGPRs, one wave per SIMD, a wave-batched inversion each): latency-bound, 1.17 ms per 8.3 M
// signatures at C4 against 0.56 ms now, 126 against 104 us at C2 (profiles/r06/finish_ab_r06.txt).
// chunked k_finish workgroup: one inversion each.  512 / 1,024 threads (fewer inversions sharing a
// CU's scalar unit) measured slower at C2 and C4: 155 / 111 us against 104 us per C2 step
// (profiles/r06/finish_ab_r06.txt)
static constexpr uint32_t FINISH_WG = 256;
template <bool ONE>
__global__ void __launch_bounds__(ONE ? 256 : FINISH_WG) k_finish(VerifyParams a) {
    const uint32_t NL = (a.gn + a.fk - 1) / a.fk;
    const uint32_t Lr = blockIdx.x * blockDim.x + threadIdx.x;
    // A wave (ONE) or a workgroup (chunked: fe_invert_block synchronizes it) with any owned lane
    // keeps all its lanes: the lanes past NL run duplicates (no writes), since every lane takes part
    // in the batched inversion and a wave with a sparse EXEC mask issues its chain 1.2-1.4x slower
    // (DESIGN.md §5.5).
    if (ONE ? (Lr & ~63u) >= NL : blockIdx.x * blockDim.x >= NL) return;
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
        // the wave's lanes share one scalar-unit inversion (ONE: <= 65,536 signatures, <= 4 waves per CU)
        const fe zi = fe_invert_batched<1>(z);
        const uint32_t f = finish_x_flags(X, zi, pf);
        if (owner) emit(i, pf, f);
    } else {
        __shared__ uint32_t inv_slot[FINISH_WG / 64][10];
        const uint32_t* zrow = a.pbuf + 10 * n;
        fe acc = fe_one();
        fe znext = load_fe_soa(zrow, n, gbase);
#pragma unroll 1
        for (uint32_t k = 0; k < cnt; ++k) {
            const size_t g = gbase + (size_t)k * NL;
            const fe z = znext;
            if (k + 1 < cnt) znext = load_fe_soa(zrow, n, g + NL);
            acc = fe_mul(acc, z);
            // the last prefix is never read back; duplicates store the owner's own values (scratch)
            if (k + 1 < cnt) store_fe_soa(a.pre, n, g, acc);
        }
        fe inv = fe_invert_block<FINISH_WG / 64>(acc, inv_slot);
#pragma unroll 1
        for (int k = (int)cnt - 1; k >= 0; --k) {
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

// One workgroup of NT threads per certificate (launch_finalize: certificates averaging more than
// 256 votes): the waves' totals meet in LDS.  Same verdicts as k_cert_finalize.
template <int NT>
__global__ void __launch_bounds__(NT) k_cert_finalize_wg(FinalizeParams a) {
    __shared__ uint32_t s_bad, s_slow, s_tsum;
    __shared__ unsigned long long s_stake;
    if (a.sig_ok) {
        const uint32_t nthr = gridDim.x * blockDim.x;
        for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < a.nsigs; v += nthr)
            a.sig_ok[v] = (a.flags[v] & NW_F_STRICT) ? 1 : 0;
    }
    const uint32_t c = blockIdx.x;   // grid = ncerts
    if (threadIdx.x == 0) {
        s_bad = s_slow = s_tsum = 0u;
        s_stake = 0ull;
    }
    __syncthreads();
    const FinalizeAcc r = finalize_scan(a, c, threadIdx.x, NT);
    if ((threadIdx.x & 63u) == 0) {
        if (r.bad) atomicOr(&s_bad, 1u);
        if (r.slow) atomicOr(&s_slow, 1u);
        atomicAdd(&s_tsum, r.tsum);
        atomicAdd(&s_stake, (unsigned long long)r.stake);
    }
    __syncthreads();
    if (threadIdx.x == 0) finalize_decide(a, c, FinalizeAcc{s_bad != 0u, s_slow != 0u, s_tsum, (uint64_t)s_stake});
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
__global__ void __launch_bounds__(64) k_cert_tail(FinalizeParams a) {
    __shared__ uint32_t part[64][40];
    cert_tail(a, threadIdx.x, part);
}

// ------------------------------------------------------------------------------------ batch preamble
// Two launches replace the five small ones a certificate batch used to start with (status /
// sig_cert / slot-count fills, input check, certificate expansion, slot histogram): ~5 us each on
// MI355X, dominated by dispatch, not work.
//   k_prep_certs:   sig_cert = NO_CERT (a vote outside every certificate gets no verdict and no
//                   exact-path entry), the slot counts, the slow-path counter and the status word = 0.
//   k_expand_count: block b expands certificates [4 b, 4 b + 4) (fewer, by 2 or 4 waves each, when
//                   certificates are large) into sig_cert (a vote already
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

static constexpr uint32_t EXPAND_WAVES_PER_BLOCK = 4;
__global__ void __launch_bounds__(256) k_expand_count(uint32_t ncerts, uint32_t nsigs, uint32_t nkeys,
                                                      const uint32_t* cert_first, const uint32_t* cert_n,
                                                      const uint32_t* signer, uint32_t* sig_cert, uint32_t* counts,
                                                      uint32_t* status, uint32_t* cert_state, uint32_t wlog) {
    extern __shared__ uint32_t hist[];
    // 2^wlog waves per certificate: their lanes write the vote -> certificate entries side by side (a
    // thread per certificate would store 667 / 6,667 entries serially at C3 / C4; one wave, 105
    // dependent atomic rounds at C4)
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t c = blockIdx.x * (EXPAND_WAVES_PER_BLOCK >> wlog) + (w >> wlog);
    const uint32_t sub = ((w & ((1u << wlog) - 1u)) << 6) | lane, step = 64u << wlog;
    bool bad = false;
    if (c < ncerts) {
        const uint32_t f = cert_first[c], n = cert_n[c];
        bad = sub == 0 && (uint64_t)f + n > nsigs;
        const uint32_t end = (uint64_t)f + n > nsigs ? nsigs : f + n;   // clamped: k_cert_finalize rejects it
        for (uint32_t v = f + sub; v < end; v += step) {
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

// Exact path, step 2 (slow_mul in nw_verify_kernels.h) over up to 256 workgroups.
__global__ void __launch_bounds__(256) k_slow_mul(VerifyParams a) {
    __shared__ uint32_t tab[SLOW_MUL_QUADS][8][40];
    slow_mul(a, blockIdx.x, gridDim.x, tab);
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

hipError_t launch_slow_tail(const VerifyParams& p, const FinalizeParams& f, int msgmode, int key_window,
                            hipStream_t st) {
    switch (key_window) {
        case 8: return launch_slow_tail_wa<8>(p, f, msgmode, st);
        case 9: return launch_slow_tail_wa<9>(p, f, msgmode, st);
        case 12: return launch_slow_tail_wa<12>(p, f, msgmode, st);
        case 13: return launch_slow_tail_wa<13>(p, f, msgmode, st);
        case 16: return launch_slow_tail_wa<16>(p, f, msgmode, st);
        case 20: return launch_slow_tail_wa<20>(p, f, msgmode, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_finish(const VerifyParams& p, hipStream_t st) {
    if (p.gn == 0) return hipSuccess;
    if (p.fk < 1 || p.fk > (uint32_t)FINISH_K || (uint64_t)p.g0 + p.gn > p.n) return hipErrorInvalidValue;
    const uint64_t lanes = (p.gn + p.fk - 1) / p.fk;
    if (p.fk == 1) hipLaunchKernelGGL(k_finish<true>, dim3(blocks_for(lanes, 256)), dim3(256), 0, st, p);
    else hipLaunchKernelGGL(k_finish<false>, dim3(blocks_for(lanes, FINISH_WG)), dim3(FINISH_WG), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeParams& p, hipStream_t st) {
    if (p.ncerts == 0) return hipSuccess;
    if (p.ncerts <= TAIL_MAX_CERTS && p.nsigs <= 64u * 1024u) {
        hipLaunchKernelGGL(k_cert_tail, dim3(1), dim3(64), 0, st, p);
        return hipGetLastError();
    }
    const uint64_t avg_votes = p.nsigs / p.ncerts;
    if (avg_votes > 1024)
        hipLaunchKernelGGL(k_cert_finalize_wg<1024>, dim3(p.ncerts), dim3(1024), 0, st, p);
    else if (avg_votes > 256)
        hipLaunchKernelGGL(k_cert_finalize_wg<256>, dim3(p.ncerts), dim3(256), 0, st, p);
    else
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
    // waves per certificate from the average vote count (a performance choice only)
    const uint64_t avg_votes = ncerts ? nsigs / ncerts : 0;
    const uint32_t wlog = avg_votes > 512 ? 2u : (avg_votes > 128 ? 1u : 0u);
    const uint32_t nb = std::max<uint32_t>(blocks_for(ncerts, EXPAND_WAVES_PER_BLOCK >> wlog),
                                           tiles ? blocks_for(nsigs, GROUP_TILE) : 0u);
    if (nb == 0) return hipGetLastError();
    const size_t lds = counts && nkeys <= GROUP_LDS_KEYS ? (size_t)nkeys * 4 : 0;
    hipLaunchKernelGGL(k_expand_count, dim3(nb), dim3(256), lds, st, ncerts, nsigs, nkeys, first, nv, signer, sig_cert,
                       counts, status, cert_state, wlog);
    return hipGetLastError();
}

// Scan + scatter of the signer grouping whose counts k_expand_count produced.
hipError_t launch_group_scatter(uint32_t n, uint32_t nkeys, const uint32_t* signer, const uint32_t* sig_cert,
                                const uint32_t* counts, uint32_t* cursor, uint32_t* perm, uint2* pinfo,
                                hipStream_t st) {
    if (n == 0 || nkeys == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_slots, dim3(1), dim3(1024), 0, st, nkeys, counts, cursor);
    if (nkeys <= GROUP_LDS_KEYS)
        hipLaunchKernelGGL(k_scatter_slots_lds, dim3(blocks_for(n, GROUP_TILE)), dim3(256), nkeys * 8, st, n, nkeys,
                           signer, sig_cert, cursor, perm, pinfo);
    else
        hipLaunchKernelGGL(k_scatter_slots, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, nkeys, signer, sig_cert,
                           cursor, perm, pinfo);
    return hipGetLastError();
}

hipError_t launch_flags_to_ok(uint32_t n, const uint32_t* flags, uint8_t* ok, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_flags_to_ok, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, flags, ok);
    return hipGetLastError();
}

}  // namespace nw
