// Scalars modulo l = 2^252 + 27742317777372353535851937790883648493 (8 x u32 LE words).
//
// Reduction is Barrett (HAC 14.42) with base 2^32, k = 8, mu = floor(2^512 / l): it replaces
// curve25519-dalek's Scalar::from_hash / from_bytes_mod_order_wide and the
// reduced products z*s, z*h (A7).  Operand-scanning products use v_mad_u64_u32; every loop has a
// constant trip count so arrays stay in registers.
#pragma once
#include <cstdint>
#include "nw_field.h"

namespace nw {

// r[na + nb] = a[na] * b[nb]
template <int NA, int NB>
NW_HD void mulw(uint32_t r[NA + NB], const uint32_t a[NA], const uint32_t b[NB]) {
#pragma unroll
    for (int i = 0; i < NA + NB; ++i) r[i] = 0;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            uint64_t t = (uint64_t)a[i] * b[j] + r[i + j];
            t += carry;
            r[i + j] = (uint32_t)t;
            carry = (uint32_t)(t >> 32);
        }
        r[i + NB] = carry;
    }
}

// a >= b (8 words)
NW_HD bool geq8(const uint32_t a[8], const uint32_t b[8]) {
    bool gt = false, lt = false;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
        const bool undecided = !gt && !lt;
        gt = gt || (undecided && a[i] > b[i]);
        lt = lt || (undecided && a[i] < b[i]);
    }
    return !lt;
}

// r = a - b (8 words, wraps)
NW_HD void sub8(uint32_t r[8], const uint32_t a[8], const uint32_t b[8]) {
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t t = (uint64_t)a[i] - b[i] - borrow;
        r[i] = (uint32_t)t;
        borrow = (uint32_t)(t >> 63);
    }
}

NW_HD void cond_sub_l(uint32_t r[8]) {
    uint32_t t[8];
    sub8(t, r, SC_L);
    const bool ge = geq8(r, SC_L);
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = ge ? t[i] : r[i];
}

// l = 2^252 + delta (delta < 2^125) in radix 2^28, 252 = 9 x 28: delta's five limbs.
static constexpr uint32_t SC_D28[5] = {0xcf5d3ed, 0x12631a5, 0x79cd658, 0xf9dea2f, 0x14de};
static constexpr uint32_t SC_M28 = 0xfffffffu;

// bits [s, s + 32) of the 64-bit hi:lo (0 <= s < 32): one v_alignbit_b32 on the device
NW_HD uint32_t funnel_lo(uint32_t hi, uint32_t lo, int s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

// r (9 limbs, [0, 2^252)) + m * delta, m in {-1, 1}, normalised: returns the carry out of limb 8
// (the multiple of 2^252), so r + m delta = q + carry 2^252.
NW_HD int sc_add_mdelta(uint32_t q[9], const uint32_t r[9], int m) {
    int c = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int s = (int)r[k] + (k < 5 ? m * (int)SC_D28[k] : 0) + c;   // |s| < 2^29
        q[k] = (uint32_t)s & SC_M28;
        c = s >> 28;   // arithmetic: floor
    }
    return c;
}

// out = x mod l for a 512-bit x (16 LE words), by folding at 2^252 = -delta (mod l):
//   x = H 2^252 + L            ->  x = L - H delta                  (H < 2^260, H delta < 2^385)
//   H delta = H1 2^252 + L1    ->  x = L - L1 + H1 delta            (H1 < 2^133, H1 delta < 2^258)
//   L - L1 + H1 delta = r + T 2^252  (T in [-1, 64])  ->  V = r - T delta, V in (-2^132, 2^252 + 2^125)
//   then V + l, V - l or V (V is within (-l, 2l)).
// Radix 2^28 keeps every column sum below 2^60, so each of the 75 products is one v_mad_u64_u32
// into a 64-bit column accumulator, with no per-product carry (Barrett at base 2^32 took 117
// products, each with its own 64-bit carry add and register moves: ~1,300 VALU per reduction
// in k_verify against ~330 here).
NW_HD void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
    uint32_t t[19];   // x in radix 2^28; limb 18 holds bits 504..511
#pragma unroll
    for (int k = 0; k < 19; ++k) {
        const int bit = 28 * k, w = bit >> 5, s = bit & 31;
        const uint32_t v = w + 1 < 16 ? funnel_lo(x[w + 1], x[w], s) : x[w] >> s;
        t[k] = k < 18 ? v & SC_M28 : v;
    }
    // P1 = H delta, H = t[9..18]: 14 limbs (the last < 2^21)
    uint32_t p1[14];
    uint64_t acc = 0;
#pragma unroll
    for (int c = 0; c < 14; ++c) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int i = c - j;
            if (i >= 0 && i < 10) acc += (uint64_t)t[9 + i] * SC_D28[j];
        }
        p1[c] = c < 13 ? (uint32_t)acc & SC_M28 : (uint32_t)acc;
        acc >>= 28;
    }
    // P2 = H1 delta, H1 = p1[9..13]: 9 limbs + p2[9] < 2^6
    uint32_t p2[10];
    acc = 0;
#pragma unroll
    for (int c = 0; c < 9; ++c) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int i = c - j;
            if (i >= 0 && i < 5) acc += (uint64_t)p1[9 + i] * SC_D28[j];
        }
        p2[c] = (uint32_t)acc & SC_M28;
        acc >>= 28;
    }
    p2[9] = (uint32_t)acc;
    // r + T 2^252 = L - L1 + P2
    uint32_t r[9];
    int c = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int s = (int)t[k] - (int)p1[k] + (int)p2[k] + c;   // (-2^28 - 2, 2^29 + 2)
        r[k] = (uint32_t)s & SC_M28;
        c = s >> 28;
    }
    const int T = (int)p2[9] + c;
    // V = r - T delta = v + T2 2^252, T2 in {-1, 0, 1}
    uint32_t v[9];
    int64_t c64 = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int64_t s = (int64_t)r[k] - (k < 5 ? (int64_t)T * (int64_t)SC_D28[k] : 0) + c64;
        v[k] = (uint32_t)s & SC_M28;
        c64 = s >> 28;
    }
    const int T2 = (int)c64;
    // canonical: T2 = -1: V + l = v + delta;  T2 = 1: V - l = v - delta when that is >= 0, else V;
    // T2 = 0: v.  (The top bit, 2^252, is set only in the first case's carry and in the last V.)
    uint32_t vp[9], vm[9];
    const int cp = sc_add_mdelta(vp, v, 1);    // v + delta = vp + cp 2^252, cp in {0, 1}
    const int cm = sc_add_mdelta(vm, v, -1);   // v - delta = vm + cm 2^252, cm in {-1, 0}
    const bool use_p = T2 < 0, use_m = T2 > 0 && cm == 0;
    const uint32_t top = use_p ? (uint32_t)cp : (use_m ? 0u : (T2 > 0 ? 1u : 0u));
    uint32_t o[10];
#pragma unroll
    for (int k = 0; k < 9; ++k) o[k] = use_p ? vp[k] : (use_m ? vm[k] : v[k]);
    o[9] = top;
    // pack 9 limbs + bit 252 into 8 words: word w = bits [32 w, 32 w + 32)
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const int k = (32 * w) / 28, s = (32 * w) % 28;
        out[w] = (o[k] >> s) | (o[k + 1] << (28 - s));
    }
}

// out = a * b mod l  (a, b < 2^256)
NW_HD void sc_mul(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
    uint32_t x[16];
    mulw<8, 8>(x, a, b);
    sc_reduce512(out, x);
}

// out = (a * b + c) mod l  (a, b, c < 2^256)
NW_HD void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
    uint32_t x[16];
    mulw<8, 8>(x, a, b);
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint64_t t = (uint64_t)x[i] + (i < 8 ? c[i] : 0u) + carry;
        x[i] = (uint32_t)t;
        carry = (uint32_t)(t >> 32);
    }
    sc_reduce512(out, x);
}

// Signature S parsing on the reference path (ed25519::Signature::from_bytes high-3-bit check,
// then dalek check_scalar / Scalar::from_canonical_bytes): accepted iff S < l.
NW_HD bool sc_is_canonical(const uint32_t s[8]) {
    if (s[7] & 0xE0000000u) return false;
    return !geq8(s, SC_L);
}

}  // namespace nw
