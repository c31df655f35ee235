// Variable-base verification kernels for keys outside the committee key cache (see nw_msm.h).
//
// Batch path (dalek::verify_batch, the cofactorless equation with seeded z_i):
//     sum_i z_i R_i + sum_i (z_i h_i mod l) A_i - (sum_i z_i s_i mod l) B == O
// evaluated literally as a segmented Pippenger MSM over the 2n points {R_i, A_i} of every batch:
//   k_msm_prep     two lanes per signature (R / A decompressed side by side): S parse, h_i, z_i,
//                  a_i = z_i h_i mod l, signed radix-2^C digits of z_i and a_i, affine Niels entries;
//   k_msm_bucket   one wave per (batch, window, chunk of <= MSM_CH entries), four per workgroup: LDS counting sort of
//                  the chunk by |digit|, each lane accumulates an equal slice of the sorted list
//                  (runs that cross slice boundaries are merged afterwards), then the bucket
//                  reduction sum_k k S_k as per-lane running sums + a cross-lane suffix scan and a
//                  tree sum over wave shuffles (ds_bpermute / DPP);
//   k_msm_wsum     one wave per (batch, window): sum of the window's chunk partials;
//   k_msm_final    one wave per batch: sum z_i s_i (column sums + Barrett), Horner over the
//                  windows, the basepoint term by the fixed-base comb, the identity test.
// Strict path (verify_strict with a decompressed key): k_verify_var, then the shared k_finish.
#include <hip/hip_runtime.h>
#include "nw_point.h"
#include "nw_sha512.h"
#include "nw_chacha.h"
#include "nw_kernels.h"
#include "nw_core.h"
#include "nw_msm.h"
#include "nw_quad.h"

// Built as three objects (Makefile: -DNW_MSM_PART=7 / 8 / 0) so the two bucket-width instantiations
// and the rest compile in parallel: one object holding all of them took ~8 minutes.
#ifndef NW_MSM_PART
#define NW_MSM_PART 0
#endif

namespace nw {

// ------------------------------------------------------------------------------------ helpers
NW_HD void store_cached(uint32_t* dst, const ge_cached& c) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        dst[k] = c.YpX.v[k];
        dst[10 + k] = c.YmX.v[k];
        dst[20 + k] = c.Z.v[k];
        dst[30 + k] = c.T2d.v[k];
    }
}

NW_HD ge_cached load_cached(const uint32_t* src) {
    ge_cached c;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        c.YpX.v[k] = src[k];
        c.YmX.v[k] = src[10 + k];
        c.Z.v[k] = src[20 + k];
        c.T2d.v[k] = src[30 + k];
    }
    return c;
}

// Doubling without the T output (the next doubling does not read T): 7 field operations.
NW_HD ge_p3 ge_dbl_xyz(const ge_p3& p) {
    const fe xx = fe_sq(p.X);
    const fe yy = fe_sq(p.Y);
    const fe zz = fe_sq(p.Z);
    const fe zz2 = fe_add(zz, zz);
    const fe s = fe_sq(fe_add(p.X, p.Y));
    const fe yr = fe_add(yy, xx);
    const fe zr = fe_sub(yy, xx);
    const fe xr = fe_sub(s, yr);
    const fe tr = fe_sub(zz2, zr);
    ge_p3 r;
    r.X = fe_mul(xr, tr);
    r.Y = fe_mul(yr, zr);
    r.Z = fe_mul(zr, tr);
    r.T = r.X;   // not meaningful
    return r;
}

// Table-entry (halved affine Niels) form of a decompressed (Z = 1) point, 128-B layout.
NW_HD void store_niels_affine(uint32_t* dst, const ge_p3& p) {
    const ge_precomp e = ge_precomp_from_affine(p.X, p.Y);
    uint4* q = reinterpret_cast<uint4*>(dst);
    uint32_t w[32];
    precomp_to_words(e, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

// 64 signed nibble digits of k < 2^253 in [-8, 7], packed as 4-bit two's complement (no carry out).
NW_HD void recode_w4(uint32_t pk[8], const uint32_t k_in[8]) {
    int carry = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        uint32_t out = 0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int b = (int)((k_in[w] >> (4 * s)) & 15u) + carry;
            carry = (b + 8) >> 4;
            const int d = b - (carry << 4);
            out |= ((uint32_t)d & 15u) << (4 * s);
        }
        pk[w] = out;
    }
}

// k * Q for k < 2^253 (8 LE words): signed radix-16 digits, most significant first.  The multiples
// 1..8 Q (projective Niels) live in this lane's 320-word slice of global scratch, so no
// runtime-indexed register array is needed; 63 x 4 doublings (T only before an addition) and 64
// additions (digit 0 adds the identity: one instruction stream for every lane).
NW_HD ge_p3 ge_scalarmult_w4(const uint32_t k_in[8], const ge_p3& Q, uint32_t* tab) {
    const ge_cached q1 = ge_to_cached(Q);
    store_cached(tab, q1);
    ge_p3 cur = ge_dbl(Q);
    store_cached(tab + 40, ge_to_cached(cur));
#pragma nounroll
    for (int e = 3; e <= 8; ++e) {
        cur = ge_add(cur, q1);
        store_cached(tab + (e - 1) * 40, ge_to_cached(cur));
    }
    uint32_t pk[8];
    recode_w4(pk, k_in);
    ge_p3 acc = ge_identity();
#pragma nounroll
    for (int i = 0; i < 64; ++i) {
        if (i) {
            acc = ge_dbl_xyz(acc);
            acc = ge_dbl_xyz(acc);
            acc = ge_dbl_xyz(acc);
            acc = ge_dbl(acc);
        }
        const int d = ((int)pk[7]) >> 28;   // sign-extended top nibble
#pragma unroll
        for (int w = 7; w > 0; --w) pk[w] = (pk[w] << 4) | (pk[w - 1] >> 28);
        pk[0] <<= 4;
        const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
        ge_cached e = load_cached(tab + (size_t)(ad ? ad - 1 : 0) * 40);
        const uint32_t mz = lane_mask(ad == 0), mn = lane_mask(d < 0);
        e.YpX = fe_select_mask(e.YpX, fe_one(), mz);
        e.YmX = fe_select_mask(e.YmX, fe_one(), mz);
        e.Z = fe_select_mask(e.Z, fe_one(), mz);
        e.T2d = fe_select_mask(e.T2d, fe_zero(), mz);
        fe_cswap_mask(e.YpX, e.YmX, mn);
        e.T2d = fe_select_mask(e.T2d, fe_carry(fe_neg(e.T2d)), mn);
        acc = ge_add(acc, e);
    }
    return acc;
}

// ge_scalarmult_w4 with every point operation split over the 4 lanes of a quad (nw_quad.h), for a
// strict call of at most 16 signatures, where the chain (252 doublings, 64 additions) is the
// call's latency.  tab: the quad's LDS slice; the multiples 1..8 Q are kept as ge_add_quad_v
// operands (entry e, lane q: tab[e * 40 + q * 10 + k]), so a lookup reads 10 words per lane.  A
// negative digit swaps lanes 0 and 1 (Y - X <-> Y + X) and negates lane 2's T; digit 0 adds the
// identity (operands 1, 1, 0, 1).
__device__ ge_p3 ge_scalarmult_w4_quad(const uint32_t k_in[8], const ge_p3& Q, uint32_t* tab) {
    const uint32_t q = threadIdx.x & 3u;
    auto put = [&](int e, const ge_p3& p) {
        const fe v = ge_quad_operand(p);
#pragma unroll
        for (int k = 0; k < 10; ++k) tab[e * 40 + q * 10 + k] = v.v[k];
    };
    put(0, Q);
    ge_p3 cur = ge_dbl_quad(Q);
    put(1, cur);
#pragma nounroll
    for (int e = 3; e <= 8; ++e) {
        cur = ge_add_quad(cur, Q);
        put(e - 1, cur);
    }
    __syncthreads();   // one-wave block: the quad's table writes before its lanes' lookups
    uint32_t pk[8];
    recode_w4(pk, k_in);
    const fe id_op = fe_select(fe_one(), fe_zero(), q == 2u);
    ge_p3 acc = ge_identity();
#pragma nounroll
    for (int i = 0; i < 64; ++i) {
        if (i) {
            acc = ge_dbl_quad(acc);
            acc = ge_dbl_quad(acc);
            acc = ge_dbl_quad(acc);
            acc = ge_dbl_quad(acc);
        }
        const int d = ((int)pk[7]) >> 28;
#pragma unroll
        for (int w = 7; w > 0; --w) pk[w] = (pk[w] << 4) | (pk[w - 1] >> 28);
        pk[0] <<= 4;
        const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
        const uint32_t slot = (d < 0 && q < 2u) ? (q ^ 1u) : q;
        const uint32_t* src = tab + (ad ? ad - 1 : 0) * 40 + slot * 10;
        fe v;
#pragma unroll
        for (int k = 0; k < 10; ++k) v.v[k] = src[k];
        v = fe_select_mask(v, fe_carry(fe_neg(v)), lane_mask(d < 0 && q == 2u));
        v = fe_select_mask(v, id_op, lane_mask(ad == 0));
        acc = ge_add_quad_v(acc, v);
    }
    return acc;
}

// ------------------------------------------------------------------------------------ strict, uncached
// One lane per signature (generic messages): P = s B - h A with A decompressed here and h A by
// ge_scalarmult_w4; writes the same (X, Z, partial flags) record as k_verify, so k_finish completes
// the strict verdict.  Semantics are those of k_verify with a cached key (nw_core.h).
// QUAD (at most VAR_QUAD_MAX_SIGS signatures: one-wave blocks of 16 quads, at most one wave per
// SIMD of the chip): a quad per signature and ge_scalarmult_w4_quad; quads past gn run duplicates
// (full EXEC) and store nothing.  Above that the lane-per-signature kernel has the throughput.
static constexpr uint32_t VAR_QUAD_MAX_SIGS = 4096;
template <bool QUAD>
__global__ void __launch_bounds__(QUAD ? 64 : 256) k_verify_var(VerifyParams a, uint32_t* scratch) {
    __shared__ uint32_t qtab[QUAD ? 16 * 320 : 1];
    uint32_t gid;
    bool owner;
    if constexpr (QUAD) {
        const uint32_t qd = blockIdx.x * 16u + (threadIdx.x >> 2);
        owner = (threadIdx.x & 3u) == 0 && qd < a.gn;
        gid = a.g0 + qd % a.gn;
    } else {
        // fewer signatures than a wave (one strict call): the idle lanes of wave 0 run duplicates, so
        // the chain issues at the full-EXEC rate; they store only what their owner stores
        const uint32_t graw = blockIdx.x * blockDim.x + threadIdx.x;
        if (graw >= a.gn && (a.gn >= 64 || graw >= 64)) return;
        owner = graw < a.gn;
        gid = a.g0 + (owner ? graw : graw % a.gn);
    }
    const uint32_t i = gid;
    uint32_t R[8], S[8], Aw[8], h[8];
    load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
    load_w8(S, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16 + 8);
    load_w8(Aw, a.sig_keys + (size_t)i * 8);
    {
        uint32_t hw[16];
        hram_generic(hw, R, Aw, a.msg_base + a.msg_off[i], a.msg_len[i]);
        sc_reduce512(h, hw);
    }
    const bool sok = sc_is_canonical(S);
    ge_p3 A;
    const bool aok = ge_decompress(A, Aw);
    A = ge_select(A, ge_identity(), !aok);
    const bool asmall = ge_is_identity(ge_dbl(ge_dbl(ge_dbl(A))));
    const uint32_t flags = (sok ? NW_F_S_OK : 0u) | (aok ? NW_F_A_OK : 0u) | (asmall ? NW_F_A_SMALL : 0u);
    // parked by the owner only: a duplicate in another wave (QUAD, more than one block) could
    // otherwise overwrite the owner's final record (store_prec_soa writes the same row)
    uint32_t* frow = a.pbuf + (size_t)PREC_FLAGS_ROW * a.n;
    if (owner) frow[gid] = flags;
    uint32_t s_use[8], zero8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s_use[k] = sok ? S[k] : 0u;
        zero8[k] = 0u;
    }
    ge_p3 P = comb_sB_minus_hA<B_WINDOW, 0>(s_use, zero8, a.btab, nullptr);
    ge_p3 hA;
    if constexpr (QUAD) hA = ge_scalarmult_w4_quad(h, A, qtab + (threadIdx.x >> 2) * 320);
    else hA = ge_scalarmult_w4(h, A, scratch + (size_t)gid * 320);
    P = ge_add(P, ge_cached_neg(ge_to_cached(hA)));
    asm volatile("" ::: "memory");
    load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
    if (owner) store_prec_soa(a.pbuf, a.n, gid, P, verify_pflags(P, R, frow[gid]));
}

// ------------------------------------------------------------------------------------ MSM
// Two lanes per signature (side = lane & 1): both run the hash, the scalars and the recoding
// (uniform code, a few thousand instructions), and each decompresses ONE point (side 0: R, side 1:
// A).  The two pow chains (~19 k instructions each) were the lane's time: one lane per signature
// gave 977 waves for 1,024 SIMDs at the MSM leg's 62,500 signatures, each running both chains
// back to back at the lone-wave rate.
#ifndef NW_MSM_PREP_WAVES
#define NW_MSM_PREP_WAVES 2   // waves per SIMD the register allocation must allow (A/B: 1)
#endif
template <int C>
__global__ void __launch_bounds__(256, NW_MSM_PREP_WAVES) k_msm_prep(MsmParams a) {
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = gt >> 1, side = gt & 1u;
    if (i >= a.nsig) return;   // both lanes of a pair leave together
    const uint32_t b = a.sig_batch[i];
    const uint32_t f = a.bfirst[b], n = a.bcount[b], t = i - f;
    uint32_t R[8], S[8], Aw[8], h[8];
    load_w8(R, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16);
    load_w8(S, reinterpret_cast<const uint32_t*>(a.sig) + (size_t)i * 16 + 8);
    load_w8(Aw, a.keys + (size_t)i * 8);
    {
        uint32_t hw[16];
        const bool fixed = a.msg_flen != ~0ull;
        const uint64_t mo = fixed ? (uint64_t)i * a.msg_flen : a.msg_off[i];
        hram_generic(hw, R, Aw, a.msg_base + mo, fixed ? a.msg_flen : a.msg_len[i]);
        sc_reduce512(h, hw);
    }
    const bool sok = sc_is_canonical(S);
    uint32_t Yw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) Yw[k] = side ? Aw[k] : R[k];
    ge_p3 Pt;
    const bool pok = ge_decompress(Pt, Yw);
    const bool qok = __shfl_xor(pok ? 1 : 0, 1, 64) != 0;   // the pair's other point
    const bool ok = sok && pok && qok;
    if (!ok && side == 0) atomicOr(&a.bad[b], 1u);
    uint32_t z4[4];
    const uint64_t bidx = a.batch_base + b;
    chacha20_z(z4, a.zseed, t + a.z_off, (uint32_t)bidx, (uint32_t)(bidx >> 32), 0u);
    uint32_t z8[8] = {z4[0], z4[1], z4[2], z4[3], 0u, 0u, 0u, 0u};
    uint32_t ks[8];
    if (side) {
        sc_mul(ks, z8, h);   // a_i = z_i h_i mod l
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) ks[k] = z8[k];
        uint32_t zs[12];
        mulw<4, 8>(zs, z4, S);
#pragma unroll
        for (int k = 0; k < 12; ++k) a.zs[(size_t)k * a.nsig + i] = ok ? zs[k] : 0u;
    }
    const size_t e = 2 * (size_t)f + (side ? n : 0u) + t;   // R entries, then the batch's A entries
    if (ok) store_niels_affine(a.ent + e * MSM_ENT_WORDS, Pt);
    const size_t E = 2 * (size_t)a.nsig;
    constexpr int NA = msm_nwin_a(C), NR = msm_nwin_r(C);
    int carry = 0;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        const int d = next_digit<C>(ks, carry);
        if (side || j < NR) a.dig[(size_t)j * E + e] = (int16_t)(ok ? d : 0);
    }
}

// Tasks per k_msm_bucket workgroup, one per wave.  With one-wave workgroups the dispatcher left
// some SIMDs with several bucket waves and others with none (per-wave timestamps: the same
// 1,953-entry accumulation took 146 k to 2.1 M cycles); a 4-wave workgroup spreads over the CU's
// four SIMDs.
#ifndef MSM_BUCKET_WAVES
#define MSM_BUCKET_WAVES 4
#endif

template <int C>
__global__ void __launch_bounds__(64 * MSM_BUCKET_WAVES) k_msm_bucket(MsmParams a) {
    constexpr uint32_t B = 1u << (C - 1);   // buckets: digit magnitudes 1..B
    constexpr uint32_t SPL = B / 64;          // buckets per lane in the reduction
    static_assert(SPL >= 1, "at least one bucket per lane");
    __shared__ uint32_t idx_w[MSM_BUCKET_WAVES][MSM_CH];
    __shared__ uint32_t cur_w[MSM_BUCKET_WAVES][B];
    __shared__ int32_t s_hb_w[MSM_BUCKET_WAVES][64];
    __shared__ uint32_t s_thru_w[MSM_BUCKET_WAVES][64];
    // one task per wave; the waves of a block only share the block (no barrier couples them)
    const uint32_t wv = threadIdx.x >> 6, L = threadIdx.x & 63u;
    const uint32_t tix = blockIdx.x * MSM_BUCKET_WAVES + wv;
    if (tix >= a.ntasks) return;
    uint32_t* idx = idx_w[wv];
    uint32_t* cur = cur_w[wv];
    int32_t* s_hb = s_hb_w[wv];
    uint32_t* s_thru = s_thru_w[wv];
    const MsmTask task = a.tasks[tix];
    const size_t E = 2 * (size_t)a.nsig;
    const int16_t* dg = a.dig + (size_t)task.win * E + task.e0;
    const uint32_t m = task.e1 - task.e0;   // <= MSM_CH (host-checked)
    for (uint32_t k = L; k < B; k += 64) cur[k] = 0;
    wave_lds_sync();
    // 1. histogram of |digit|
    for (uint32_t e = L; e < m; e += 64) {
        const int d = dg[e];
        if (d) atomicAdd(&cur[(uint32_t)(d < 0 ? -d : d) - 1u], 1u);
    }
    wave_lds_sync();
    // 2. exclusive scan: lane L owns buckets [L SPL, L SPL + SPL)
    uint32_t loc[SPL];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t s = 0; s < SPL; ++s) {
        loc[s] = cur[L * SPL + s];
        sum += loc[s];
    }
    uint32_t inc = sum;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off, 64);
        if (L >= off) inc += v;
    }
    const uint32_t total = __shfl(inc, 63, 64);
    uint32_t run = inc - sum;
    wave_lds_sync();
#pragma unroll
    for (uint32_t s = 0; s < SPL; ++s) {
        cur[L * SPL + s] = run;   // cursor; after the scatter it is the bucket's end position
        run += loc[s];
    }
    wave_lds_sync();
    // 3. scatter: (bucket << 16) | (negative << 15) | entry offset
    for (uint32_t e = L; e < m; e += 64) {
        const int d = dg[e];
        if (d) {
            const uint32_t k = (uint32_t)(d < 0 ? -d : d) - 1u;
            const uint32_t pos = atomicAdd(&cur[k], 1u);
            idx[pos] = (k << 16) | (d < 0 ? 0x8000u : 0u) | e;
        }
    }
    wave_lds_sync();
    // 4. balanced accumulation: lane L takes sorted positions [p0, p1)
    const uint32_t q = (total + 63) / 64;
    const uint32_t p0 = min(total, L * q), p1 = min(total, p0 + q);
    uint32_t* bk = a.bkt + (size_t)tix * B * MSM_PT_WORDS;
    uint32_t* hp = a.part + (size_t)tix * 128 * MSM_PT_WORDS;   // head partials [64][40]
    uint32_t* tp = hp + 64 * MSM_PT_WORDS;                               // tail partials [64][40]
    const uint32_t* ent = a.ent + (size_t)task.e0 * MSM_ENT_WORDS;
    int32_t hb = -1, tb = -1;
    uint32_t thru = 0;
    if (p0 < p1) {
        ge_p3 acc = ge_identity();
        uint32_t cb = idx[p0] >> 16;
        bool head = p0 > 0 && (idx[p0 - 1] >> 16) == cb;
        uint32_t v = idx[p0];
        // the entry's halves are loaded in the order the digit's sign needs (load_ent_sw): no
        // select between the gather and the products
        ent_sw nx = load_ent_sw(ent + (size_t)(v & 0x7FFFu) * MSM_ENT_WORDS, (v & 0x8000u) != 0);
#pragma nounroll
        for (uint32_t p = p0; p < p1; ++p) {
            const ent_sw cur = nx;
            const bool neg = (v & 0x8000u) != 0;
            const uint32_t vn = p + 1 < p1 ? idx[p + 1] : v;
            if (p + 1 < p1)   // prefetch the next entry under this addition
                nx = load_ent_sw(ent + (size_t)(vn & 0x7FFFu) * MSM_ENT_WORDS, (vn & 0x8000u) != 0);
            // fused-carry product groups: two waves share each SIMD here (412 vs 424 us per launch)
            acc = ge_madd_sgn<true>(acc, ent_sw_precomp(cur), lane_mask(neg));
            const bool last = p + 1 == p1;
            const bool brk = last || (vn >> 16) != cb;   // the run of bucket cb ends here
            if (brk) {
                const bool tail = last && p1 < total && (idx[p1] >> 16) == cb;
                if (head) {
                    store_p3(hp + L * MSM_PT_WORDS, acc);
                    hb = (int32_t)cb;
                    thru = tail ? 1u : 0u;
                } else if (tail) {
                    store_p3(tp + L * MSM_PT_WORDS, acc);
                    tb = (int32_t)cb;
                } else {
                    store_p3(bk + cb * MSM_PT_WORDS, acc);   // complete run: the whole bucket
                }
                acc = ge_identity();
                head = false;
                cb = vn >> 16;
            }
            v = vn;
        }
    }
    s_hb[L] = hb;
    s_thru[L] = thru;
    wave_lds_sync();
    // 5. merge runs that cross slice boundaries: the lane holding a bucket's first entry adds the
    //    head partials of the following lanes (through-partials continue the chain)
    if (tb >= 0) {
        ge_p3 acc = load_p3(tp + L * MSM_PT_WORDS);
#pragma nounroll
        for (uint32_t k = L + 1; k < 64; ++k) {
            if (s_hb[k] != tb) break;
            acc = ge_add_p3(acc, load_p3(hp + k * MSM_PT_WORDS));
            if (!s_thru[k]) break;
        }
        store_p3(bk + (uint32_t)tb * MSM_PT_WORDS, acc);
    }
    wave_lds_sync();
    // 6. bucket reduction sum_k k S_k (k = magnitude).  Lane L: W_L = sum_s (s+1) S_{L SPL + s},
    //    T_L = sum_s S_{L SPL + s};  total = sum_L W_L + SPL * sum_{L >= 1} U_L with the suffix sums
    //    U_L = sum_{L' >= L} T_L'.
    ge_p3 T = ge_identity(), W = ge_identity();
#pragma unroll
    for (int s = (int)SPL - 1; s >= 0; --s) {
        const uint32_t k = L * SPL + (uint32_t)s;
        const uint32_t start = k ? cur[k - 1] : 0u;
        const bool empty = cur[k] == start;
        const ge_p3 Sk = ge_select(load_p3(bk + k * MSM_PT_WORDS), ge_identity(), empty);
        T = ge_add_p3(T, Sk);
        W = ge_add_p3(W, T);
    }
    ge_p3 U = T;
#pragma unroll
    for (unsigned off = 1; off < 64; off <<= 1) {
        const ge_p3 V = ge_shfl_down(U, off);
        const ge_p3 Us = ge_add_p3(U, V);
        U = ge_select(U, Us, L + off < 64);
    }
#pragma unroll
    for (uint32_t s = 1; s < SPL; s <<= 1) U = ge_dbl(U);
    ge_p3 X = ge_select(W, ge_add_p3(W, U), L >= 1);
#pragma unroll
    for (unsigned off = 32; off > 0; off >>= 1) {
        const ge_p3 V = ge_shfl_down(X, off);
        X = ge_add_p3(X, V);   // lanes >= off add garbage; only lane 0's result is used
    }
    if (L == 0) store_p3(a.wpart + (size_t)task.out * MSM_PT_WORDS, X);
}

// One wave per (batch, window): sum of the window's chunk partials into slot wfirst[bw].
template <int C>
__global__ void __launch_bounds__(64) k_msm_wsum(MsmParams a, uint32_t* wsum) {
    const uint32_t bw = blockIdx.x, L = threadIdx.x;
    const uint32_t w0 = a.wfirst[bw], w1 = a.wfirst[bw + 1];
    ge_p3 acc = ge_identity();
    for (uint32_t w = w0 + L; w < w1; w += 64) acc = ge_add_p3(acc, load_p3(a.wpart + (size_t)w * MSM_PT_WORDS));
    // only the levels that the partial count needs (lanes >= w1 - w0 hold the identity)
    const uint32_t m = w1 - w0;
#pragma unroll
    for (unsigned off = 32; off > 0; off >>= 1)
        if (off < m) acc = ge_add_p3(acc, ge_shfl_down(acc, off));
    if (L == 0) store_p3(wsum + (size_t)bw * MSM_PT_WORDS, acc);
}

template <int C>
__global__ void __launch_bounds__(64) k_msm_final(MsmParams a, const uint32_t* wsum) {
    constexpr int NA = msm_nwin_a(C);
    const uint32_t b = blockIdx.x, L = threadIdx.x;
    const uint32_t f = a.bfirst[b], n = a.bcount[b];
    uint64_t col[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) col[k] = 0;
    for (uint32_t t = L; t < n; t += 64) {
#pragma unroll
        for (int k = 0; k < 12; ++k) col[k] += a.zs[(size_t)k * a.nsig + f + t];
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) {
#pragma unroll
        for (unsigned off = 32; off > 0; off >>= 1) col[k] += __shfl_xor(col[k], off, 64);
    }
    // every lane runs the serial tail (the values are VGPR-resident, see ge_to_vgpr); lane 0 stores
    // sum_i z_i s_i < n 2^381 < 2^413: 16 words, then mod l
    uint32_t x[16];
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t v = (k < 12 ? col[k] : 0ull) + carry;
        x[k] = (uint32_t)v;
        carry = v >> 32;
    }
    uint32_t bc[8];
    sc_reduce512(bc, x);
    ge_p3 acc = ge_to_vgpr(load_p3(wsum + ((size_t)b * NA + NA - 1) * MSM_PT_WORDS));
#pragma nounroll
    for (int j = NA - 2; j >= 0; --j) {
#pragma unroll
        for (int c = 0; c < C; ++c) acc = ge_dbl_quad(acc);
        acc = ge_add_quad(acc, load_p3(wsum + ((size_t)b * NA + j) * MSM_PT_WORDS));
    }
    uint32_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const ge_p3 PB = comb_sB_minus_hA<B_WINDOW, 0>(bc, zero8, a.btab, nullptr);
    acc = ge_add(acc, ge_cached_neg(ge_to_cached(PB)));
    if (L != 0) return;
    if (a.point_out) store_p3(a.point_out + (size_t)b * MSM_PT_WORDS, acc);
    if (a.batch_ok) a.batch_ok[b] = (!a.bad[b] && ge_is_identity(acc)) ? 1 : 0;
}

// Sum of npts extended points (the shards of one split batch) == identity.
#if NW_MSM_PART == 0
__global__ void __launch_bounds__(64) k_points_identity(uint32_t npts, const uint32_t* pts, uint8_t* out) {
    // lanes stride over the points, then a shuffle tree (all values in VGPRs)
    const uint32_t L = threadIdx.x;
    ge_p3 acc = ge_to_vgpr(ge_identity());
    for (uint32_t k = L; k < npts; k += 64) acc = ge_add_p3(acc, load_p3(pts + (size_t)k * MSM_PT_WORDS));
#pragma unroll
    for (unsigned off = 32; off > 0; off >>= 1) acc = ge_add_p3(acc, ge_shfl_down(acc, off));
    if (L == 0) out[0] = ge_is_identity(acc) ? 1 : 0;
}
#endif

template <int C>
hipError_t launch_msm_c(const MsmParams& p, hipStream_t st) {
    hipError_t e = hipSuccess;
    // no signatures (an empty shard of a split batch, counts all 0): the bad flags are zeroed by
    // the metadata upload and no zs column is read, so wsum/final give the identity -> Ok, as
    // dalek's empty batch
    if (p.nsig) {
        hipLaunchKernelGGL(k_msm_prep<C>, dim3(blocks_for(2 * (uint64_t)p.nsig, 256)), dim3(256), 0, st, p);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (p.ntasks) {
        hipLaunchKernelGGL(k_msm_bucket<C>, dim3((p.ntasks + MSM_BUCKET_WAVES - 1) / MSM_BUCKET_WAVES),
                           dim3(64 * MSM_BUCKET_WAVES), 0, st, p);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    constexpr int NA = msm_nwin_a(C);
    // window sums live after the task partials in wpart; batches of up to MSM_CH / 2 signatures have
    // one task per window, whose partial is already the window sum (the launch was ~48 us of shuffle
    // levels adding identities)
    uint32_t* wsum = p.wpart;
    if (!p.one_task_windows) {
        wsum = p.wpart + (size_t)p.ntasks * MSM_PT_WORDS;
        hipLaunchKernelGGL(k_msm_wsum<C>, dim3(p.nb * NA), dim3(64), 0, st, p, wsum);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_msm_final<C>, dim3(p.nb), dim3(64), 0, st, p, (const uint32_t*)wsum);
    return hipGetLastError();
}

#if NW_MSM_PART == 7 || NW_MSM_PART == 8
template hipError_t launch_msm_c<NW_MSM_PART>(const MsmParams&, hipStream_t);
#else
extern template hipError_t launch_msm_c<7>(const MsmParams&, hipStream_t);
extern template hipError_t launch_msm_c<8>(const MsmParams&, hipStream_t);

hipError_t launch_msm(const MsmParams& p, hipStream_t st) {
    if (p.nb == 0) return hipSuccess;
    switch (p.c) {
        case 7: return launch_msm_c<7>(p, st);
        case 8: return launch_msm_c<8>(p, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_msm_points_identity(uint32_t npts, const uint32_t* pts, uint8_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_points_identity, dim3(1), dim3(64), 0, st, npts, pts, out);
    return hipGetLastError();
}

hipError_t launch_verify_var(const VerifyParams& p, int msgmode, uint32_t* scratch, hipStream_t st) {
    if (p.gn == 0) return hipSuccess;
    if (msgmode != 1) return hipErrorInvalidValue;
    if (p.gn <= VAR_QUAD_MAX_SIGS)
        hipLaunchKernelGGL(k_verify_var<true>, dim3((p.gn + 15) / 16), dim3(64), 0, st, p, scratch);
    else hipLaunchKernelGGL(k_verify_var<false>, dim3(blocks_for(p.gn, 256)), dim3(256), 0, st, p, scratch);
    return hipGetLastError();
}
#endif  // NW_MSM_PART

}  // namespace nw
