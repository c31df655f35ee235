// GF(2^255 - 19) arithmetic for gfx950.
//
// Representation: 10 x u32 limbs, radix 2^25.5 (limb widths 26,25,26,25,...; limb i sits at
// bit offset ceil(25.5 i)).  Products use u32 x u32 -> u64 multiply-accumulate, which hipcc
// lowers to v_mad_u64_u32 (measured on MI355X: 2.9e13 lane-MAD/s chip-wide, about half the
// simple-VALU rate; profiles/r01_valu_peak.json).  Ten independent u64 column accumulators
// give the scheduler ILP; the carry chain interleaves two halves (0..4 / 5..9).
//
// Limb-size discipline ("k" = limbs <= k * 2^26 even / k * 2^25 odd):
//   * tight (k ~ 1): output of fe_mul / fe_sq / fe_sub / fe_carry / fe_frombytes
//   * fe_add of two tight values: k = 2;  one more add: k = 3
//   * fe_mul(h, f, g) requires k_g <= 3 (19*g must fit 32 bits) and k_f * k_g <= 32
//     (u64 column sums stay below 2^64); every call site below respects k <= 3.
//   * fe_sub(h, f, g) requires k_g <= 3 (uses f + 4p - g) and returns a tight value.
// The same functions compile for the host (``__host__``) so tools/ can unit-test them
// against the Python oracle; the shipped library only ever runs them on the GPU.
#pragma once
#include <cstdint>
#include "nw_constants.h"

#define NW_HD __host__ __device__ __forceinline__

namespace nw {

struct fe {
    uint32_t v[10];
};

static constexpr uint32_t M26 = (1u << 26) - 1;
static constexpr uint32_t M25 = (1u << 25) - 1;

NW_HD fe fe_from_const(const uint32_t c[10]) {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = c[i];
    return r;
}

NW_HD fe fe_zero() {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = 0;
    return r;
}

NW_HD fe fe_one() {
    fe r = fe_zero();
    r.v[0] = 1;
    return r;
}

NW_HD fe fe_add(const fe& f, const fe& g) {
    fe h;
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
    return h;
}

// One carry pass over u32 limbs (inputs up to ~2^31); result tight.
NW_HD void fe_carry_inplace(fe& h) {
    uint32_t c;
    c = h.v[0] >> 26; h.v[1] += c; h.v[0] &= M26;
    c = h.v[5] >> 25; h.v[6] += c; h.v[5] &= M25;
    c = h.v[1] >> 25; h.v[2] += c; h.v[1] &= M25;
    c = h.v[6] >> 26; h.v[7] += c; h.v[6] &= M26;
    c = h.v[2] >> 26; h.v[3] += c; h.v[2] &= M26;
    c = h.v[7] >> 25; h.v[8] += c; h.v[7] &= M25;
    c = h.v[3] >> 25; h.v[4] += c; h.v[3] &= M25;
    c = h.v[8] >> 26; h.v[9] += c; h.v[8] &= M26;
    c = h.v[4] >> 26; h.v[5] += c; h.v[4] &= M26;
    c = h.v[9] >> 25; h.v[0] += 19u * c; h.v[9] &= M25;
    c = h.v[0] >> 26; h.v[1] += c; h.v[0] &= M26;
    c = h.v[5] >> 25; h.v[6] += c; h.v[5] &= M25;
}

NW_HD fe fe_carry(const fe& f) {
    fe h = f;
    fe_carry_inplace(h);
    return h;
}

// h = f - g  (k_g <= 3), tight output.
NW_HD fe fe_sub(const fe& f, const fe& g) {
    fe h;
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + FE_4P[i] - g.v[i];
    fe_carry_inplace(h);
    return h;
}

// h = f - g without the carry pass (k_f <= 1, g <= 4p limb-wise): limbs < 1.25 * 2^28 / 2^27,
// i.e. k = 5.  Only valid as the FIRST operand of fe_mul with a second operand of k <= 6/... such
// that k_f * k_g <= 32 (see the limb-size discipline above): 5 x 1 and 5 x 2 are used.
NW_HD fe fe_sub_loose(const fe& f, const fe& g) {
    fe h;
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + FE_4P[i] - g.v[i];
    return h;
}

// h = f - g without the carry pass for tight f and g (g limbs <= 2p limbs): f + 2p - g, limbs
// < 3 * 2^26 (k = 3): still a valid second fe_mul operand (19 * 3 * 2^26 < 2^32).
NW_HD fe fe_sub2p_loose(const fe& f, const fe& g) {
    fe h;
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + FE_2P[i] - g.v[i];
    return h;
}

// h = -f for tight f, k = 2 output (no carry): 2p - f.
NW_HD fe fe_neg(const fe& f) {
    fe h;
#pragma unroll
    for (int i = 0; i < 10; ++i) h.v[i] = FE_2P[i] - f.v[i];
    return h;
}

// Reduce 10 u64 column sums to tight u32 limbs.
NW_HD fe fe_reduce_wide(uint64_t h[10]) {
    uint64_t c;
    c = h[0] >> 26; h[1] += c; h[0] &= M26;
    c = h[4] >> 26; h[5] += c; h[4] &= M26;
    c = h[1] >> 25; h[2] += c; h[1] &= M25;
    c = h[5] >> 25; h[6] += c; h[5] &= M25;
    c = h[2] >> 26; h[3] += c; h[2] &= M26;
    c = h[6] >> 26; h[7] += c; h[6] &= M26;
    c = h[3] >> 25; h[4] += c; h[3] &= M25;
    c = h[7] >> 25; h[8] += c; h[7] &= M25;
    c = h[4] >> 26; h[5] += c; h[4] &= M26;
    c = h[8] >> 26; h[9] += c; h[8] &= M26;
    c = h[9] >> 25; h[0] += c * 19u; h[9] &= M25;
    c = h[0] >> 26; h[1] += c; h[0] &= M26;
    fe r;
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = (uint32_t)h[i];
    return r;
}

// 2x as an addition: on gfx950 v_add_u32 issues at the full rate, the v_lshlrev_b32 the compiler
// picks for 2 * x at half rate (profiles/r01/isa/isa_rates_vop2.jsonl).  Off by default: it removes
// 35 of 1,264 VALU instructions per comb step but measured no faster at C2 (k_verify 1.188 vs
// 1.181 ms, profiles/r02/ab_r02d.txt) — the loop is bound by v_mad_u64_u32 issue, not by these.
NW_HD uint32_t dbl32(uint32_t x) {
    return 2u * x;
}

// Fused-carry product scanning (the mixed addition's products, ge_madd).  Column k of h = f g is
// ONE v_mad_u64_u32 chain that starts from column k-1's carry (acc = c_{k-1} + sum_i f_i g_{k-i}),
// so the carry enters as the first MAD's addend instead of a separate 64-bit add; the wrap carry
// (x19) and one 0 -> 1 carry tighten the result (limb 1 <= 2^25 + 2^18, as fe_reduce_wide).  A lone
// chain would issue one MAD per dependency latency (and gfx950 needs wait states between dependent
// 64-bit MADs), so products are only computed this way in groups whose chains interleave MAD by
// MAD: an empty asm over all accumulators after each step keeps the group in lockstep (without it
// the scheduler re-serializes the chains).  Measured on MI355X at C2 (profiles/r02/ab_r02k.txt):
// k_verify 1.176 -> 1.132 ms against operand scanning with a separate carry chain.
#ifndef NW_MADD_FUSED
#define NW_MADD_FUSED 1   // 0: k_verify's throughput kernel uses operand-scanned products too (A/B)
#endif
NW_HD fe fe_fused_wrap(uint32_t r[10], uint64_t c) {
    const uint64_t t = (uint64_t)r[0] + c * 19u;
    r[0] = (uint32_t)t & M26;
    r[1] += (uint32_t)(t >> 26);
    fe o;
#pragma unroll
    for (int i = 0; i < 10; ++i) o.v[i] = r[i];
    return o;
}

// h = f * g mod p, operand scanning: ten independent column accumulators (ILP for a lone product),
// then one carry chain.  Coefficient of f_i g_j: 2 if i, j both odd; x19 if i + j >= 10.
NW_HD fe fe_mul(const fe& f, const fe& g) {
    uint32_t g19[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) g19[j] = 19u * g.v[j];
    uint32_t f2[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) f2[i] = (i & 1) ? dbl32(f.v[i]) : f.v[i];
    uint64_t acc[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
#pragma unroll
        for (int j = 0; j < 10; ++j) {
            const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
            const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
            acc[(i + j) % 10] += (uint64_t)a * b;
        }
    }
    return fe_reduce_wide(acc);
}

// Two independent products h1 = f1 g1, h2 = f2 g2 as two interleaved fused-carry chains.
NW_HD void fe_mul2(fe& h1, const fe& f1, const fe& g1, fe& h2, const fe& f2, const fe& g2) {
    uint32_t g19a[10], f2a[10], g19b[10], f2b[10], ra[10], rb[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        g19a[j] = 19u * g1.v[j];
        g19b[j] = 19u * g2.v[j];
        f2a[j] = (j & 1) ? dbl32(f1.v[j]) : f1.v[j];
        f2b[j] = (j & 1) ? dbl32(f2.v[j]) : f2.v[j];
    }
    uint64_t ca = 0, cb = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint64_t acca = ca, accb = cb;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int j = (k - i + 10) % 10;
            const bool dbl = (i & 1) && (j & 1), wrap = i + j >= 10;
            acca += (uint64_t)(dbl ? f2a[i] : f1.v[i]) * (wrap ? g19a[j] : g1.v[j]);
            accb += (uint64_t)(dbl ? f2b[i] : f2.v[i]) * (wrap ? g19b[j] : g2.v[j]);
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+v"(acca), "+v"(accb));
#endif
        }
        const uint32_t m = (k & 1) ? M25 : M26;
        const int sh = (k & 1) ? 25 : 26;
        ra[k] = (uint32_t)acca & m;
        rb[k] = (uint32_t)accb & m;
        ca = acca >> sh;
        cb = accb >> sh;
    }
    h1 = fe_fused_wrap(ra, ca);
    h2 = fe_fused_wrap(rb, cb);
}

// Three independent products as three interleaved fused-carry chains (NW_MADD3: the mixed
// addition's first half a, b, c in one group).
NW_HD void fe_mul3(fe& h1, const fe& f1, const fe& g1, fe& h2, const fe& f2, const fe& g2, fe& h3, const fe& f3,
                   const fe& g3) {
    uint32_t a19[10], b19[10], c19[10], fa[10], fb[10], fc[10], r1[10], r2[10], r3[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        a19[j] = 19u * g1.v[j];
        b19[j] = 19u * g2.v[j];
        c19[j] = 19u * g3.v[j];
        fa[j] = (j & 1) ? dbl32(f1.v[j]) : f1.v[j];
        fb[j] = (j & 1) ? dbl32(f2.v[j]) : f2.v[j];
        fc[j] = (j & 1) ? dbl32(f3.v[j]) : f3.v[j];
    }
    uint64_t c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint64_t x1 = c1, x2 = c2, x3 = c3;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int j = (k - i + 10) % 10;
            const bool dbl = (i & 1) && (j & 1), wrap = i + j >= 10;
            x1 += (uint64_t)(dbl ? fa[i] : f1.v[i]) * (wrap ? a19[j] : g1.v[j]);
            x2 += (uint64_t)(dbl ? fb[i] : f2.v[i]) * (wrap ? b19[j] : g2.v[j]);
            x3 += (uint64_t)(dbl ? fc[i] : f3.v[i]) * (wrap ? c19[j] : g3.v[j]);
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+v"(x1), "+v"(x2), "+v"(x3));
#endif
        }
        const uint32_t m = (k & 1) ? M25 : M26;
        const int sh = (k & 1) ? 25 : 26;
        r1[k] = (uint32_t)x1 & m;
        r2[k] = (uint32_t)x2 & m;
        r3[k] = (uint32_t)x3 & m;
        c1 = x1 >> sh;
        c2 = x2 >> sh;
        c3 = x3 >> sh;
    }
    h1 = fe_fused_wrap(r1, c1);
    h2 = fe_fused_wrap(r2, c2);
    h3 = fe_fused_wrap(r3, c3);
}

// The four products of the mixed addition's second half, X = e f, Y = g h, Z = g f, T = e h, as
// four interleaved fused-carry chains (dependent MADs 4 apart: no wait states; 19 f, 19 h and the
// doubled odd limbs of e and g are each computed once).
NW_HD void fe_mul4_efgh(fe& X, fe& Y, fe& Z, fe& T, const fe& e, const fe& f, const fe& g, const fe& h) {
    uint32_t f19[10], h19[10], e2[10], g2[10], rx[10], ry[10], rz[10], rt[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        f19[j] = 19u * f.v[j];
        h19[j] = 19u * h.v[j];
        e2[j] = (j & 1) ? dbl32(e.v[j]) : e.v[j];
        g2[j] = (j & 1) ? dbl32(g.v[j]) : g.v[j];
    }
    uint64_t cx = 0, cy = 0, cz = 0, ct = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint64_t ax = cx, ay = cy, az = cz, at = ct;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int j = (k - i + 10) % 10;
            const bool dbl = (i & 1) && (j & 1), wrap = i + j >= 10;
            const uint32_t ei = dbl ? e2[i] : e.v[i], gi = dbl ? g2[i] : g.v[i];
            const uint32_t fj = wrap ? f19[j] : f.v[j], hj = wrap ? h19[j] : h.v[j];
            ax += (uint64_t)ei * fj;
            ay += (uint64_t)gi * hj;
            az += (uint64_t)gi * fj;
            at += (uint64_t)ei * hj;
#if defined(__HIP_DEVICE_COMPILE__)
            asm volatile("" : "+v"(ax), "+v"(ay), "+v"(az), "+v"(at));
#endif
        }
        const uint32_t m = (k & 1) ? M25 : M26;
        const int sh = (k & 1) ? 25 : 26;
        rx[k] = (uint32_t)ax & m; ry[k] = (uint32_t)ay & m; rz[k] = (uint32_t)az & m; rt[k] = (uint32_t)at & m;
        cx = ax >> sh; cy = ay >> sh; cz = az >> sh; ct = at >> sh;
    }
    X = fe_fused_wrap(rx, cx);
    Y = fe_fused_wrap(ry, cy);
    Z = fe_fused_wrap(rz, cz);
    T = fe_fused_wrap(rt, ct);
}

// h = f^2 mod p (55 products).
NW_HD fe fe_sq(const fe& f) {
    uint64_t acc[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[k] = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
#pragma unroll
        for (int j = i; j < 10; ++j) {
            uint32_t m1 = (i == j) ? 1u : 2u;
            if ((i & 1) && (j & 1)) m1 *= 2u;
            const uint32_t a = f.v[i] * m1;
            const uint32_t b = (i + j >= 10) ? 19u * f.v[j] : f.v[j];
            acc[(i + j) % 10] += (uint64_t)a * b;
        }
    }
    return fe_reduce_wide(acc);
}

NW_HD fe fe_sqn(fe f, int n) {
#pragma nounroll
    for (int i = 0; i < n; ++i) f = fe_sq(f);
    return f;
}

// z^(2^252 - 3) = z^((p-5)/8)
NW_HD fe fe_pow22523(const fe& z) {
    fe t0 = fe_sq(z);                  // 2
    fe t1 = fe_sqn(t0, 2);             // 8
    t1 = fe_mul(z, t1);                // 9
    t0 = fe_mul(t0, t1);               // 11
    t0 = fe_sq(t0);                    // 22
    t0 = fe_mul(t1, t0);               // 31 = 2^5 - 1
    t1 = fe_sqn(t0, 5);
    t0 = fe_mul(t1, t0);               // 2^10 - 1
    t1 = fe_sqn(t0, 10);
    t1 = fe_mul(t1, t0);               // 2^20 - 1
    fe t2 = fe_sqn(t1, 20);
    t1 = fe_mul(t2, t1);               // 2^40 - 1
    t1 = fe_sqn(t1, 10);
    t0 = fe_mul(t1, t0);               // 2^50 - 1
    t1 = fe_sqn(t0, 50);
    t1 = fe_mul(t1, t0);               // 2^100 - 1
    t2 = fe_sqn(t1, 100);
    t1 = fe_mul(t2, t1);               // 2^200 - 1
    t1 = fe_sqn(t1, 50);
    t0 = fe_mul(t1, t0);               // 2^250 - 1
    t0 = fe_sqn(t0, 2);                // 2^252 - 4
    return fe_mul(t0, z);              // 2^252 - 3
}

// z^(p-2) = z^(2^255 - 21)
NW_HD fe fe_invert(const fe& z) {
    fe t0 = fe_sq(z);                  // 2
    fe t1 = fe_sqn(t0, 2);             // 8
    t1 = fe_mul(z, t1);                // 9
    t0 = fe_mul(t0, t1);               // 11
    fe t2 = fe_sq(t0);                 // 22
    t1 = fe_mul(t1, t2);               // 31
    t2 = fe_sqn(t1, 5);
    t1 = fe_mul(t2, t1);               // 2^10 - 1
    t2 = fe_sqn(t1, 10);
    t2 = fe_mul(t2, t1);               // 2^20 - 1
    fe t3 = fe_sqn(t2, 20);
    t2 = fe_mul(t3, t2);               // 2^40 - 1
    t2 = fe_sqn(t2, 10);
    t1 = fe_mul(t2, t1);               // 2^50 - 1
    t2 = fe_sqn(t1, 50);
    t2 = fe_mul(t2, t1);               // 2^100 - 1
    t3 = fe_sqn(t2, 100);
    t2 = fe_mul(t3, t2);               // 2^200 - 1
    t2 = fe_sqn(t2, 50);
    t1 = fe_mul(t2, t1);               // 2^250 - 1
    t1 = fe_sqn(t1, 5);                // 2^255 - 32
    return fe_mul(t1, t0);             // 2^255 - 21
}

// Canonical little-endian 8 x u32 words of f mod p.
NW_HD void fe_tobytes_w(uint32_t out[8], const fe& fin) {
    fe h = fe_carry(fin);
    fe_carry_inplace(h);
    // q = floor((V + 19) / 2^255) in {0, 1}
    uint32_t q = (h.v[0] + 19u) >> 26;
    q = (h.v[1] + q) >> 25;
    q = (h.v[2] + q) >> 26;
    q = (h.v[3] + q) >> 25;
    q = (h.v[4] + q) >> 26;
    q = (h.v[5] + q) >> 25;
    q = (h.v[6] + q) >> 26;
    q = (h.v[7] + q) >> 25;
    q = (h.v[8] + q) >> 26;
    q = (h.v[9] + q) >> 25;
    h.v[0] += 19u * q;
    uint32_t c;
    c = h.v[0] >> 26; h.v[1] += c; h.v[0] &= M26;
    c = h.v[1] >> 25; h.v[2] += c; h.v[1] &= M25;
    c = h.v[2] >> 26; h.v[3] += c; h.v[2] &= M26;
    c = h.v[3] >> 25; h.v[4] += c; h.v[3] &= M25;
    c = h.v[4] >> 26; h.v[5] += c; h.v[4] &= M26;
    c = h.v[5] >> 25; h.v[6] += c; h.v[5] &= M25;
    c = h.v[6] >> 26; h.v[7] += c; h.v[6] &= M26;
    c = h.v[7] >> 25; h.v[8] += c; h.v[7] &= M25;
    c = h.v[8] >> 26; h.v[9] += c; h.v[8] &= M26;
    h.v[9] &= M25;   // drops 2^255 (q*p subtraction)
    // pack: offsets 0,26,51,77,102,128,153,179,204,230
    out[0] = h.v[0] | (h.v[1] << 26);
    out[1] = (h.v[1] >> 6) | (h.v[2] << 19);
    out[2] = (h.v[2] >> 13) | (h.v[3] << 13);
    out[3] = (h.v[3] >> 19) | (h.v[4] << 6);
    out[4] = h.v[5] | (h.v[6] << 25);
    out[5] = (h.v[6] >> 7) | (h.v[7] << 19);
    out[6] = (h.v[7] >> 13) | (h.v[8] << 12);
    out[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}

// 8 LE words -> limbs (bit 255 ignored; values >= p are kept as a non-canonical representative,
// exactly like curve25519-dalek FieldElement::from_bytes).
NW_HD fe fe_frombytes_w(const uint32_t w[8]) {
    fe h;
    h.v[0] = w[0] & M26;
    h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;
    h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;
    h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;
    h.v[4] = (w[3] >> 6) & M26;
    h.v[5] = w[4] & M25;
    h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;
    h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;
    h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;
    h.v[9] = (w[7] >> 6) & M25;
    return h;
}

NW_HD bool fe_iszero(const fe& f) {
    uint32_t w[8];
    fe_tobytes_w(w, f);
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) a |= w[i];
    return a == 0;
}

NW_HD bool fe_isnegative(const fe& f) {
    uint32_t w[8];
    fe_tobytes_w(w, f);
    return (w[0] & 1u) != 0;
}

NW_HD bool fe_eq(const fe& f, const fe& g) {
    return fe_iszero(fe_sub(f, g));
}

// All-ones / zero lane mask from a predicate.  On the device the mask is hidden from the optimizer
// so that the xor/and selects below stay bit operations (v_bfi_b32 / v_bitop3_b32) instead of
// being recognised as selects and lowered to v_cndmask_b32 (a dependent chain of which issues at
// 11 cycles per wave64 instruction on gfx950, profiles/r01/isa/isa_rates_vop2.jsonl).  A/B on
// MI355X at C2 (profiles/r01_ab_select.txt): k_verify 1.214 ms vs 1.230 ms with cndmask selects.
NW_HD uint32_t lane_mask(bool b) {
    uint32_t m = 0u - (uint32_t)b;
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(m));
#endif
    return m;
}

NW_HD fe fe_select_mask(const fe& a, const fe& b, uint32_t m) {
    fe r;
#pragma unroll
    for (int i = 0; i < 10; ++i) r.v[i] = a.v[i] ^ ((a.v[i] ^ b.v[i]) & m);
    return r;
}

NW_HD fe fe_select(const fe& a, const fe& b, bool take_b) {
    return fe_select_mask(a, b, lane_mask(take_b));
}

// (a, b) <- (b, a) where m is all-ones: 3 bit operations per limb pair.
NW_HD void fe_cswap_mask(fe& a, fe& b, uint32_t m) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t t = (a.v[i] ^ b.v[i]) & m;
        a.v[i] ^= t;
        b.v[i] ^= t;
    }
}

// curve25519-dalek FieldElement::sqrt_ratio_i (see oracle/ed25519_oracle.py sqrt_ratio_i).
NW_HD bool fe_sqrt_ratio_i(fe& r_out, const fe& u, const fe& v) {
    const fe v3 = fe_mul(fe_sq(v), v);
    const fe v7 = fe_mul(fe_sq(v3), v);
    fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
    const fe check = fe_mul(v, fe_sq(r));
    const fe neg_u = fe_neg(u);
    const fe sqm1 = fe_from_const(FE_SQRTM1);
    const bool correct = fe_eq(check, u);
    const bool flipped = fe_eq(check, neg_u);
    const bool flipped_i = fe_eq(check, fe_mul(neg_u, sqm1));
    r = fe_select(r, fe_mul(r, sqm1), flipped || flipped_i);
    r = fe_select(r, fe_carry(fe_neg(r)), fe_isnegative(r));
    r_out = r;
    return correct || flipped;
}

}  // namespace nw
