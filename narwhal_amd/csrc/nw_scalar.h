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

// out = x mod l for a 512-bit x (16 LE words).
NW_HD void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
    uint32_t q1[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) q1[i] = x[7 + i];
    uint32_t q2[18];
    mulw<9, 9>(q2, q1, SC_MU);
    uint32_t q3[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) q3[i] = q2[9 + i];
    // r2 = (q3 * l) mod 2^288 : only the low 9 words are needed
    uint32_t r2[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) r2[i] = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (i + j < 9) {
                uint64_t t = (uint64_t)q3[i] * SC_L[j] + r2[i + j];
                t += carry;
                r2[i + j] = (uint32_t)t;
                carry = (uint32_t)(t >> 32);
            }
        }
        if (i + 8 < 9) r2[i + 8] += carry;
    }
    // r = x mod 2^288 - r2 (mod 2^288); result < 3l
    uint32_t r[9];
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const uint64_t t = (uint64_t)x[i] - r2[i] - borrow;
        r[i] = (uint32_t)t;
        borrow = (uint32_t)(t >> 63);
    }
    // r < 3l < 2^255: word 8 is zero
    uint32_t r8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r8[i] = r[i];
    cond_sub_l(r8);
    cond_sub_l(r8);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = r8[i];
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
