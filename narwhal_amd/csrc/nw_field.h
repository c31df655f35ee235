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
#ifndef NW_ADD_DBL
#define NW_ADD_DBL 0
#endif
NW_HD uint32_t dbl32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && NW_ADD_DBL
    uint32_t r;
    asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
#else
    return 2u * x;
#endif
}

// Product scanning with the carry fused into the next column (NW_FUSED_CARRY, experimental):
// column k's multiply-accumulate chain starts from the carry out of column k-1, so the carry
// needs no separate 64-bit add; the wrap carry (x19) and one 0 -> 1 carry tighten the result.
// Same bounds as fe_reduce_wide (limb 1 <= 2^25 + 2^18).
#ifndef NW_FUSED_CARRY
#define NW_FUSED_CARRY 0
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

// h = f * g mod p.  Coefficient of f_i g_j: 2 if i, j both odd; x19 if i + j >= 10.
NW_HD fe fe_mul(const fe& f, const fe& g) {
#if NW_FUSED_CARRY
    uint32_t g19[10], f2[10], r[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) g19[j] = 19u * g.v[j];
#pragma unroll
    for (int i = 0; i < 10; ++i) f2[i] = (i & 1) ? dbl32(f.v[i]) : f.v[i];
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint64_t acc = c;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int j = (k - i + 10) % 10;
            const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
            const uint32_t b = (i + j >= 10) ? g19[j] : g.v[j];
            acc += (uint64_t)a * b;
        }
        r[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
        c = acc >> ((k & 1) ? 25 : 26);
    }
    return fe_fused_wrap(r, c);
#else
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
#endif
}

// h = f^2 mod p (55 products).
NW_HD fe fe_sq(const fe& f) {
#if NW_FUSED_CARRY
    uint32_t r[10];
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint64_t acc = c;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const int j = (k - i + 10) % 10;
            if (j < i) continue;   // each unordered pair once
            uint32_t m1 = (i == j) ? 1u : 2u;
            if ((i & 1) && (j & 1)) m1 *= 2u;
            const uint32_t a = f.v[i] * m1;
            const uint32_t b = (i + j >= 10) ? 19u * f.v[j] : f.v[j];
            acc += (uint64_t)a * b;
        }
        r[k] = (uint32_t)acc & ((k & 1) ? M25 : M26);
        c = acc >> ((k & 1) ? 25 : 26);
    }
    return fe_fused_wrap(r, c);
#else
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
#endif
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
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NW_CNDMASK_SELECT)
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
