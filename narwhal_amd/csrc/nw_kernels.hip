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
// without any variable-base work; everything else goes to the exact path (k_slow_sig), which
// evaluates the remaining terms literally.  Verdicts are therefore identical to dalek's for every
// input (not just honest ones) given the same z_i.
//
// Pipeline per batch: k_expand_certs -> [signer grouping] -> k_verify (P_i, one lane per signature)
// -> k_finish (Montgomery batch inversion of Z over FINISH_K signatures per lane, encoding match,
// strict verdict) -> k_slow_sig (compacted list of mismatches only) -> k_cert_finalize.
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
    load_w8(Aw, a.keys_raw + (size_t)slot * 8);
    kinfo = a.key_info[slot];
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
// One lane per signature: P_i = s_i B - h_i A_i, written as (X, Y, Z) to pbuf; partial flags
// (S ok, A ok, A small, torsion coefficient for torsion keys).
#ifdef NW_VERIFY_WAVES
#define NW_VERIFY_BOUNDS __launch_bounds__(256, NW_VERIFY_WAVES)
#else
#define NW_VERIFY_BOUNDS __launch_bounds__(256)
#endif
template <int MSGMODE, int WA>
__global__ void NW_VERIFY_BOUNDS k_verify(VerifyParams a) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= a.n) return;
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
    a.flags[i] = flags;
    const ge_p3 P = compute_P<WA>(S, h, sok, a.btab, a.key_tab + (size_t)slot * comb_words(WA));
    // P in processing order, struct-of-arrays (column gid): coalesced for k_finish
    store_xyz_soa(a.pbuf, a.n, gid, P);
}

// ------------------------------------------------------------------------------------ signer grouping
// Counting sort of signature indices by key-cache slot: perm lists the signatures of slot 0, then
// slot 1, ...  (order inside a slot is arbitrary; every output is written at the original index).
// Committees are small next to a batch (100 keys, 1M signatures), so global per-slot atomics would
// serialize: each workgroup histograms a GROUP_TILE-signature tile in LDS and touches global
// memory once per (tile, slot).  Above GROUP_LDS_KEYS slots the plain global-atomic form is used
// (contention is then spread over many addresses anyway).
static constexpr uint32_t GROUP_TILE = 4096;
static constexpr uint32_t GROUP_LDS_KEYS = 8192;

__global__ void __launch_bounds__(256) k_count_slots(uint32_t n, const uint32_t* signer, uint32_t* counts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&counts[signer[i]], 1u);
}

__global__ void __launch_bounds__(256) k_count_slots_lds(uint32_t n, uint32_t nkeys, const uint32_t* signer,
                                                         uint32_t* counts) {
    extern __shared__ uint32_t hist[];
    for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * GROUP_TILE;
    const uint32_t t1 = min(n, t0 + GROUP_TILE);
    for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) atomicAdd(&hist[signer[i]], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x)
        if (hist[k]) atomicAdd(&counts[k], hist[k]);
}

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

__global__ void __launch_bounds__(256) k_scatter_slots(uint32_t n, const uint32_t* signer, uint32_t* cursor,
                                                       uint32_t* perm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) perm[atomicAdd(&cursor[signer[i]], 1u)] = i;
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
    for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) atomicAdd(&base[signer[i]], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nkeys; k += blockDim.x)
        if (base[k]) base[k] = atomicAdd(&cursor[k], base[k]);
    __syncthreads();
    for (uint32_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
        const uint32_t k = signer[i];
        perm[base[k] + atomicAdd(&rank[k], 1u)] = i;
    }
}

// ------------------------------------------------------------------------------------ finish
// Montgomery batch inversion of the Z of FINISH_K signatures per lane (one field inversion per
// chunk), affine x, y, encoding match against R, strict verdict, and (batch mode) compaction of the
// mismatching signatures into the exact-path list.  Lane L of NL owns the processing-order columns
// g = L, L + NL, L + 2 NL, ... so every pbuf / pre access of a wave is one contiguous 256-B run.
__global__ void __launch_bounds__(256) k_finish(VerifyParams a) {
    const uint32_t NL = (a.n + FINISH_K - 1) / FINISH_K;
    const uint32_t L = blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= NL) return;
    const uint32_t cnt = (a.n - L + NL - 1) / NL;   // columns L + k NL < n
    const size_t n = a.n;
    // Both chains are fully unrolled over FINISH_K (guarded by cnt) so the column loads are
    // independent of the running products and issue ahead of them: with one wave per SIMD the
    // kernel is latency-bound, and a load inside the serial chain would stall it every step.
    fe acc = fe_one();
#pragma unroll
    for (int k = 0; k < FINISH_K; ++k) {
        if ((uint32_t)k < cnt) {
            const size_t g = L + (size_t)k * NL;
            acc = fe_mul(acc, load_fe_soa(a.pbuf + 20 * n, n, g));
            store_fe_soa(a.pre, n, g, acc);
        }
    }
    fe inv = fe_invert_sg(acc);
#pragma unroll
    for (int k = FINISH_K - 1; k >= 0; --k) {
        if ((uint32_t)k < cnt) {
            const size_t g = L + (size_t)k * NL;
            fe zi = inv;
            if (k > 0) {
                zi = fe_mul(inv, load_fe_soa(a.pre, n, g - NL));
                inv = fe_mul(inv, load_fe_soa(a.pbuf + 20 * n, n, g));
            }
            const uint32_t i = a.perm ? a.perm[g] : (uint32_t)g;
            uint32_t R[8];
            load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
            uint32_t f = finish_flags(load_fe_soa(a.pbuf, n, g), load_fe_soa(a.pbuf + 10 * n, n, g), zi, R,
                                      a.flags[i]);
            if (a.batch_mode && (f & (NW_F_S_OK | NW_F_A_OK)) == (NW_F_S_OK | NW_F_A_OK) && !(f & NW_F_MATCH)) {
                f |= NW_F_SLOW;
                const uint32_t t = atomicAdd(a.slow_count, 1u);
                a.slow_list[t] = i;
                a.slow_slot[i] = t;
            }
            a.flags[i] = f;
        }
    }
}

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

// Per-certificate verdict: definitive Err on any bad S / undecodable A / undecodable R, else the
// exact remaining batch sum (usually empty) must be the identity.  One 64-lane wave per
// certificate: lanes stride over the votes (coalesced flag reads), wave reductions combine them;
// the exact sum over slow-path terms (failing certificates only) runs on lane 0.
__global__ void __launch_bounds__(256) k_cert_finalize(FinalizeParams a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c >= a.ncerts) return;   // whole wave exits together
    const uint32_t first = a.cert_first[c], nv = a.cert_n[c];
    bool bad = false, slow = false;
    uint32_t tsum = 0;
    uint64_t stake = 0;
    for (uint32_t v = lane; v < nv; v += 64) {
        const uint32_t f = a.flags[first + v];
        bad = bad || ((f & (NW_F_S_OK | NW_F_A_OK)) != (NW_F_S_OK | NW_F_A_OK)) || (f & NW_F_R_BAD);
        slow = slow || (f & NW_F_SLOW);
        tsum += (f >> NW_F_TCOEF_SHIFT) & 7u;
        if (f & NW_F_STRICT) stake += a.stake[a.signer[first + v]];
    }
    bad = __any(bad);
    slow = __any(slow);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        tsum += __shfl_xor(tsum, off, 64);
        stake += __shfl_xor(stake, off, 64);
    }
    if (lane != 0) return;
    bool ok;
    if (bad) {
        ok = false;
    } else if (!slow) {
        ok = (tsum & 7u) == 0;
    } else {
        ge_p3 acc = ge_identity();
        for (uint32_t v = 0; v < nv; ++v) {
            const uint32_t f = a.flags[first + v];
            if (f & NW_F_SLOW) {
                const ge_p3 Q = load_p3(a.slow_buf + (size_t)a.slow_slot[first + v] * SLOW_WORDS);
                acc = ge_add(acc, ge_to_cached(Q));
            }
        }
        const ge_cached t8c = ge_to_cached(ge_t8());
        for (uint32_t k = 0; k < (tsum & 7u); ++k) acc = ge_add(acc, t8c);
        ok = ge_is_identity(acc);
    }
    if (a.cert_ok) a.cert_ok[c] = ok ? 1 : 0;
    if (a.accepted_stake) a.accepted_stake[c] = stake;
}

__global__ void __launch_bounds__(256) k_expand_certs(uint32_t ncerts, const uint32_t* cert_first,
                                                      const uint32_t* cert_n, uint32_t* sig_cert) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncerts) return;
    const uint32_t f = cert_first[c], n = cert_n[c];
    for (uint32_t v = 0; v < n; ++v) sig_cert[f + v] = c;
}

__global__ void __launch_bounds__(256) k_flags_to_ok(uint32_t n, const uint32_t* flags, uint8_t* ok) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ok[i] = (flags[i] & NW_F_STRICT) ? 1 : 0;
}

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
__global__ void __launch_bounds__(256) k_comb_build(uint32_t nk, const uint32_t* bases, uint32_t* tab) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nch = (comb_ent(W) + COMB_CH - 1) / COMB_CH;
    const uint64_t per_key = (uint64_t)comb_pos(W) * nch;
    if (gid >= (uint64_t)nk * per_key) return;
    const uint32_t j = (uint32_t)(gid / per_key);
    const uint64_t rem = gid % per_key;
    comb_chunk_build<W, COMB_CH>(bases + (size_t)j * comb_pos(W) * 40, (uint32_t)(rem / nch), (uint32_t)(rem % nch),
                                 tab + (size_t)j * comb_words(W));
}

// ------------------------------------------------------------------------------------ SHA-512 bulk
// One lane per message (each message is an inherently sequential compression chain).
__global__ void __launch_bounds__(256) k_sha512_many(uint32_t n, const uint8_t* base, const uint64_t* off,
                                                     const uint64_t* len, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* m = base + off[i];
    const uint64_t L = len[i];
    const uint64_t nfull = L / 128;
    uint64_t st[8];
    sha512_init(st);
    uint64_t w[16];
    const bool aligned = (reinterpret_cast<uintptr_t>(m) & 3u) == 0;
    for (uint64_t b = 0; b < nfull; ++b) {
        const uint8_t* blk = m + b * 128;
        if (aligned) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(blk);
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = be64_from_le32(p[2 * k], p[2 * k + 1]);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                uint64_t x = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) x = (x << 8) | blk[8 * k + j];
                w[k] = x;
            }
        }
        sha512_compress(st, w);
    }
    // tail: remaining bytes + padding (1 or 2 blocks)
    const uint64_t rem = L - nfull * 128;
    const uint8_t* tail = m + nfull * 128;
    const int tb = rem + 17 <= 128 ? 1 : 2;
    for (int b = 0; b < tb; ++b) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint64_t x = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t p = (uint64_t)b * 128 + 8 * k + j;
                const uint32_t byte = p < rem ? tail[p] : (p == rem ? 0x80u : 0u);
                x = (x << 8) | byte;
            }
            w[k] = x;
        }
        if (b == tb - 1) {
            w[14] = L >> 61;
            w[15] = L << 3;
        }
        sha512_compress(st, w);
    }
    uint32_t d[16];
    sha512_digest_le32(d, st);
    uint4* o = reinterpret_cast<uint4*>(out + (size_t)i * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = make_uint4(d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]);
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

// ------------------------------------------------------------------------------------ launchers
static inline unsigned blocks_for(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

template <int MSGMODE>
static void launch_verify_w(const VerifyParams& p, int wa, bool slow, uint32_t n_upper, hipStream_t st) {
    const dim3 b(256);
    const dim3 g(blocks_for(slow ? n_upper : p.n, 256));
    switch (wa) {
        case 8:
            if (slow) hipLaunchKernelGGL((k_slow_sig<MSGMODE, 8>), g, b, 0, st, p);
            else hipLaunchKernelGGL((k_verify<MSGMODE, 8>), g, b, 0, st, p);
            break;
        case 12:
            if (slow) hipLaunchKernelGGL((k_slow_sig<MSGMODE, 12>), g, b, 0, st, p);
            else hipLaunchKernelGGL((k_verify<MSGMODE, 12>), g, b, 0, st, p);
            break;
        case 16:
            if (slow) hipLaunchKernelGGL((k_slow_sig<MSGMODE, 16>), g, b, 0, st, p);
            else hipLaunchKernelGGL((k_verify<MSGMODE, 16>), g, b, 0, st, p);
            break;
        default:
            if (slow) hipLaunchKernelGGL((k_slow_sig<MSGMODE, 20>), g, b, 0, st, p);
            else hipLaunchKernelGGL((k_verify<MSGMODE, 20>), g, b, 0, st, p);
            break;
    }
}

static hipError_t launch_vs(const VerifyParams& p, int msgmode, int key_window, bool slow, uint32_t n_upper,
                            hipStream_t st) {
    if (key_window != 8 && key_window != 12 && key_window != 16 && key_window != 20) return hipErrorInvalidValue;
    if (msgmode == 0)
        launch_verify_w<0>(p, key_window, slow, n_upper, st);
    else
        launch_verify_w<1>(p, key_window, slow, n_upper, st);
    return hipGetLastError();
}

hipError_t launch_verify(const VerifyParams& p, int msgmode, int key_window, hipStream_t st) {
    if (p.n == 0) return hipSuccess;
    return launch_vs(p, msgmode, key_window, false, 0, st);
}

hipError_t launch_group_by_signer(uint32_t n, uint32_t nkeys, const uint32_t* signer, uint32_t* counts,
                                  uint32_t* cursor, uint32_t* perm, hipStream_t st) {
    if (n == 0 || nkeys == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(counts, 0, (size_t)nkeys * 4, st);
    if (e != hipSuccess) return e;
    const bool lds = nkeys <= GROUP_LDS_KEYS;
    if (lds)
        hipLaunchKernelGGL(k_count_slots_lds, dim3(blocks_for(n, GROUP_TILE)), dim3(256), nkeys * 4, st, n, nkeys,
                           signer, counts);
    else
        hipLaunchKernelGGL(k_count_slots, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, signer, counts);
    hipLaunchKernelGGL(k_scan_slots, dim3(1), dim3(1024), 0, st, nkeys, counts, cursor);
    if (lds)
        hipLaunchKernelGGL(k_scatter_slots_lds, dim3(blocks_for(n, GROUP_TILE)), dim3(256), nkeys * 8, st, n, nkeys,
                           signer, cursor, perm);
    else
        hipLaunchKernelGGL(k_scatter_slots, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, signer, cursor, perm);
    return hipGetLastError();
}

hipError_t launch_finish(const VerifyParams& p, hipStream_t st) {
    if (p.n == 0) return hipSuccess;
    const uint64_t lanes = (p.n + FINISH_K - 1) / FINISH_K;
    hipLaunchKernelGGL(k_finish, dim3(blocks_for(lanes, 256)), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_slow(const VerifyParams& p, int msgmode, int key_window, uint32_t n_upper, hipStream_t st) {
    if (n_upper == 0) return hipSuccess;
    return launch_vs(p, msgmode, key_window, true, n_upper, st);
}

hipError_t launch_finalize(const FinalizeParams& p, hipStream_t st) {
    if (p.ncerts == 0) return hipSuccess;
    hipLaunchKernelGGL(k_cert_finalize, dim3(blocks_for((uint64_t)p.ncerts * 64, 256)), dim3(256), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_expand_certs(uint32_t ncerts, const uint32_t* first, const uint32_t* nv, uint32_t* sig_cert,
                               hipStream_t st) {
    if (ncerts == 0) return hipSuccess;
    hipLaunchKernelGGL(k_expand_certs, dim3(blocks_for(ncerts, 256)), dim3(256), 0, st, ncerts, first, nv,
                       sig_cert);
    return hipGetLastError();
}

hipError_t launch_flags_to_ok(uint32_t n, const uint32_t* flags, uint8_t* ok, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_flags_to_ok, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, flags, ok);
    return hipGetLastError();
}

template <int W>
static hipError_t launch_key_prep_w(uint32_t nk, const uint32_t* keys_raw, uint32_t* key_info, uint32_t* bases,
                                    uint32_t* tab, hipStream_t st) {
    hipLaunchKernelGGL(k_key_prep<W>, dim3(blocks_for(nk, 64)), dim3(64), 0, st, nk, keys_raw, key_info, bases);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t total = (uint64_t)nk * comb_pos(W) * ((comb_ent(W) + COMB_CH - 1) / COMB_CH);
    hipLaunchKernelGGL(k_comb_build<W>, dim3(blocks_for(total, 256)), dim3(256), 0, st, nk, bases, tab);
    return hipGetLastError();
}

hipError_t launch_key_prep(uint32_t nk, const uint32_t* keys_raw, uint32_t* key_info, uint32_t* bases,
                           uint32_t* tab, int window, hipStream_t st) {
    if (nk == 0) return hipSuccess;
    switch (window) {
        case 8: return launch_key_prep_w<8>(nk, keys_raw, key_info, bases, tab, st);
        case 12: return launch_key_prep_w<12>(nk, keys_raw, key_info, bases, tab, st);
        case 16: return launch_key_prep_w<16>(nk, keys_raw, key_info, bases, tab, st);
        case 20: return launch_key_prep_w<20>(nk, keys_raw, key_info, bases, tab, st);
        case B_WINDOW: return launch_key_prep_w<B_WINDOW>(nk, keys_raw, key_info, bases, tab, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_sha512_many(uint32_t n, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                              uint8_t* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sha512_many, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, base, off, len, out);
    return hipGetLastError();
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
