// edwards25519 group arithmetic for gfx950 (twisted Edwards, a = -1).
//
//   ge_p3      extended (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z
//   ge_precomp affine Niels, HALVED ((y+x)/2, (y-x)/2, d xy): fixed-base table entries and MSM
//              bucket entries, 7M mixed addition (see ge_madd for why halved)
//   ge_cached  projective Niels (Y+X, Y-X, Z, 2dT): variable-base operands, 8M addition
//
// All formulas are the complete unified ones (Hisil-Wong-Carter-Dawson 2008), so results are the
// exact group elements curve25519-dalek computes for any decodable input, torsion included.
#pragma once
#include "nw_field.h"
#include "nw_inv.h"
#include "nw_scalar.h"

namespace nw {

struct ge_p3 {
    fe X, Y, Z, T;
};
struct ge_precomp {
    fe ypx, ymx, xy2d;
};
struct ge_cached {
    fe YpX, YmX, Z, T2d;
};

// Table entry layout in HBM: 32 u32 words = 128 B (one cache line):
//   [0..9] (y+x)/2, [10..11] zero, [12..21] (y-x)/2, [22..31] d x y, radix-2^25.5 limbs as words.
// (y+x)/2 and (y-x)/2 both start 16-byte aligned, so a comb step loads them in either order by
// address: the conditional negation of a signed digit (-q swaps the two and negates d x y) costs no
// select between the gather and the first products (comb_pass_dig; the sign of d x y is applied
// to the product T d x y instead, ge_madd_sgn, or taken from the negated copy of the table,
// k_comb_negate).  Round 4's layout ([0..9] [10..19] [20..29], pad) needed the entry whole before
// 30 selects.
// A packed variant (round 5): [0..7] (y+x)/2, [8..15] (y-x)/2, [16..23] d x y as canonical
// 255-bit words, [24..31] unused: a gather touches 96 of the 128 bytes and unpacks the limbs after
// the load (fe_frombytes_w, ~46 VALU per comb step).  Measured at C2 (profiles/r05/kverify_ab_r05.txt):
// k_verify 1.092-1.113 ms packed vs 1.093-1.119 ms unpacked, i.e. no gain for 4% more VALU per
// wave, so the unpacked layout stays the default.
static constexpr int ENT_YPX = 0, ENT_YMX = 12, ENT_XY2D = 22;
static constexpr int PRECOMP_WORDS = 32;
// Fixed-base combs: signed radix-2^W digits, one table per digit position holding the multiples
// |d| * 2^(W*pos) * P for |d| = 0..2^(W-1) (0 = identity).  W = 24 for the basepoint (11 positions,
// 11.8 GB, shared by every signature: HBM-resident by design, 288 GB per GPU); W = 8 / 12 / 16 / 20
// for committee keys, chosen by committee size so the key cache fits its HBM budget
// (nw_opts.key_window).  Additions per scalar = ceil(256 / W); no doublings.
NW_HD constexpr int comb_pos(int w) { return (256 + w - 1) / w; }
NW_HD constexpr int comb_ent(int w) { return (1 << (w - 1)) + 1; }
NW_HD constexpr size_t comb_words(int w) { return (size_t)comb_pos(w) * comb_ent(w) * PRECOMP_WORDS; }
#ifndef NW_BW
#define NW_BW 24
#endif
static constexpr int B_WINDOW = NW_BW;
// NW_BASE_NEGTAB (variant builds): the basepoint table carries its negated copy too (+11.8 GB at W24),
// so the basepoint pass also picks entries by address.  Measured in shader cycles per C2 k_verify launch
// (PMC GRBM_GUI_ACTIVE, profiles/r05/pmc_ab_r05.txt): 2.00-2.14 M without the copy against 2.07-2.27 M
// with it; the doubled table costs more than the 30 selects per basepoint step it saves.
#ifndef NW_BASE_NEGTAB
#define NW_BASE_NEGTAB 0
#endif
static constexpr bool B_NEGTAB = NW_BASE_NEGTAB;
static constexpr int B_TABLES = B_NEGTAB ? 2 : 1;

NW_HD ge_p3 ge_identity() {
    ge_p3 r;
    r.X = fe_zero();
    r.Y = fe_one();
    r.Z = fe_one();
    r.T = fe_zero();
    return r;
}

NW_HD ge_precomp ge_precomp_identity() {
    ge_precomp r;
    r.ypx = fe_from_const(FE_HALF);
    r.ymx = fe_from_const(FE_HALF);
    r.xy2d = fe_zero();
    return r;
}

#ifndef NW_MADD3
#define NW_MADD3 1   // with the digits in LDS (k_verify): a, b, c as one three-way fused group
#endif
// p + q (mixed, halved entry).  The HWCD formulas with every quantity halved: A/2 = (Y1-X1)(y-x)/2,
// B/2, C/2 = T1 d x y, D/2 = Z1 (no doubling), E/2, F/2 = Z1 - C/2, G/2, H/2; the products
// E F, G H, G F, E H are the sum times 1/4 in every coordinate, i.e. the same projective point.
// Halving the table entries once at build time removes the 2 Z1 addition and the carry pass of F
// from every addition: F/2 = Z1 + 2p - C/2 has limbs < 3 * 2^26 (k = 3), so it is a valid second
// fe_mul operand (19 F/2 < 2^32) without carrying.  Limb budget: (Y1+X1) k=2, (Y1-X1) and
// e = b - a loose (k = 5, first operands only), f k=3, g = Z1 + C/2 k=2, h = b + a k=2; products
// e f 15, g h 4, g f 6, e h 10 <= 32.  xy2d (d x y) may be k=2 (negated entry).
// The two halves of the mixed addition: a, b, c and the sums e, f, g, h; then the four products.
struct madd_mid {
    fe e, f, g, h;
};

// FUSED selects the fused-carry product groups (fe_mul2 / fe_mul4_efgh).  They pay off only where
// several waves share a SIMD (k_verify's throughput kernel, 3 waves): at one wave per SIMD the
// lockstep chains expose their MAD latency and the operand-scanned products are faster (worker
// chunks, k_verify<1,W>: 98 vs 62-85 M sigs/s; profiles/r02/ab_r02.txt r02t).
template <bool FUSED>
NW_HD madd_mid ge_madd_s1(const ge_p3& p, const ge_precomp& q) {
    madd_mid m;
    if constexpr (FUSED && NW_MADD3) {
        fe a, b, c;
        fe_mul3(a, fe_sub_loose(p.Y, p.X), q.ymx, b, fe_add(p.Y, p.X), q.ypx, c, p.T, q.xy2d);
        m.e = fe_sub_loose(b, a);
        m.h = fe_add(b, a);
        m.f = fe_sub2p_loose(p.Z, c);
        m.g = fe_add(p.Z, c);
    } else if constexpr (FUSED) {
        // a and b as one interleaved pair; c alone by operand scanning (a lone fused chain stalls);
        // used when the three-way group does not fit the register budget
        fe a, b;
        fe_mul2(a, fe_sub_loose(p.Y, p.X), q.ymx, b, fe_add(p.Y, p.X), q.ypx);
        const fe c = fe_mul(p.T, q.xy2d);
        m.e = fe_sub_loose(b, a);
        m.h = fe_add(b, a);
        m.f = fe_sub2p_loose(p.Z, c);
        m.g = fe_add(p.Z, c);
    } else {
        const fe a = fe_mul(fe_sub_loose(p.Y, p.X), q.ymx);
        const fe b = fe_mul(fe_add(p.Y, p.X), q.ypx);
        const fe c = fe_mul(p.T, q.xy2d);
        m.e = fe_sub_loose(b, a);
        m.h = fe_add(b, a);
        m.f = fe_sub2p_loose(p.Z, c);
        m.g = fe_add(p.Z, c);
    }
    return m;
}

template <bool FUSED>
NW_HD ge_p3 ge_madd_s2(const madd_mid& m) {
    ge_p3 r;
    if constexpr (FUSED) {
        fe_mul4_efgh(r.X, r.Y, r.Z, r.T, m.e, m.f, m.g, m.h);
    } else {
        r.X = fe_mul(m.e, m.f);
        r.Y = fe_mul(m.g, m.h);
        r.Z = fe_mul(m.g, m.f);
        r.T = fe_mul(m.e, m.h);
    }
    return r;
}

template <bool FUSED = false>
NW_HD ge_p3 ge_madd(const ge_p3& p, const ge_precomp& q) { return ge_madd_s2<FUSED>(ge_madd_s1<FUSED>(p, q)); }

// p + (q or -q) for an entry whose (y+x)/2 and (y-x)/2 were already swapped when negated (loaded in
// that order, load_ent_sw) and whose d x y was NOT: the sign lands on the product c = T d x y
// instead.  -q's f and g are q's g and f (F/2 = Z - C/2, G/2 = Z + C/2 with C negated), so with the
// mask m all-ones f = Z + c and g = Z + 2p - c (k = 3: g feeds fe_mul4_efgh as a first operand
// against h, k = 2, and f, k <= 3: products 6 and 9 <= 32).
template <bool FUSED>
NW_HD madd_mid ge_madd_s1_sgn(const ge_p3& p, const ge_precomp& q, uint32_t m) {
    madd_mid r;
    fe a, b, c;
    if constexpr (FUSED && NW_MADD3) {
        fe_mul3(a, fe_sub_loose(p.Y, p.X), q.ymx, b, fe_add(p.Y, p.X), q.ypx, c, p.T, q.xy2d);
    } else if constexpr (FUSED) {
        fe_mul2(a, fe_sub_loose(p.Y, p.X), q.ymx, b, fe_add(p.Y, p.X), q.ypx);
        c = fe_mul(p.T, q.xy2d);
    } else {
        a = fe_mul(fe_sub_loose(p.Y, p.X), q.ymx);
        b = fe_mul(fe_add(p.Y, p.X), q.ypx);
        c = fe_mul(p.T, q.xy2d);
    }
    r.e = fe_sub_loose(b, a);
    r.h = fe_add(b, a);
    const fe fq = fe_sub2p_loose(p.Z, c), gq = fe_add(p.Z, c);
    r.f = fe_select_mask(fq, gq, m);
    r.g = fe_select_mask(gq, fq, m);
    return r;
}

template <bool FUSED = false>
NW_HD ge_p3 ge_madd_sgn(const ge_p3& p, const ge_precomp& q, uint32_t m) {
    return ge_madd_s2<FUSED>(ge_madd_s1_sgn<FUSED>(p, q, m));
}

// The chain's last addition: X, Y, Z only (T = e h is not needed by k_verify's checks; the rare
// lane that parks P for the exact path rescales instead, p3_from_xyz).  Saves one of the 162 FMs.
template <bool FUSED>
NW_HD ge_p3 ge_madd_s2_xyz(const madd_mid& m) {
    ge_p3 r;
    if constexpr (FUSED) {
        fe_mul3(r.X, m.e, m.f, r.Y, m.g, m.h, r.Z, m.g, m.f);
    } else {
        r.X = fe_mul(m.e, m.f);
        r.Y = fe_mul(m.g, m.h);
        r.Z = fe_mul(m.g, m.f);
    }
    r.T = fe_zero();   // not computed
    return r;
}

// (X : Y : Z) -> extended (X Z : Y Z : Z^2 : X Y), the same point with T = X Y / Z.
NW_HD ge_p3 p3_from_xyz(const ge_p3& p) {
    ge_p3 r;
    r.X = fe_mul(p.X, p.Z);
    r.Y = fe_mul(p.Y, p.Z);
    r.Z = fe_sq(p.Z);
    r.T = fe_mul(p.X, p.Y);
    return r;
}

// Extended point of a halved affine Niels entry, with no field multiplication beyond T:
// X = (y+x)/2 - (y-x)/2 = x, Y = y, Z = 1, T = xy = (d x y) / d.
// Starts a comb chain without the 7-multiplication addition to the identity.
NW_HD ge_p3 ge_from_precomp(const ge_precomp& q) {
    ge_p3 r;
    r.X = fe_sub(q.ypx, q.ymx);
    r.Y = fe_carry(fe_add(q.ypx, q.ymx));
    r.Z = fe_one();
    r.T = fe_mul(q.xy2d, fe_from_const(FE_INVD));
    return r;
}

// Table-entry form of affine (x, y) (tight limbs): halved affine Niels.
NW_HD ge_precomp ge_precomp_from_affine(const fe& x, const fe& y) {
    ge_precomp q;
    const fe half = fe_from_const(FE_HALF);
    q.ypx = fe_mul(fe_add(y, x), half);
    q.ymx = fe_mul(fe_sub(y, x), half);
    q.xy2d = fe_mul(fe_mul(x, y), fe_from_const(FE_D));
    return q;
}

NW_HD ge_cached ge_to_cached(const ge_p3& p) {
    ge_cached c;
    c.YpX = fe_carry(fe_add(p.Y, p.X));
    c.YmX = fe_sub(p.Y, p.X);
    c.Z = p.Z;
    c.T2d = fe_mul(p.T, fe_from_const(FE_D2));
    return c;
}

NW_HD ge_cached ge_cached_neg(const ge_cached& q) {
    ge_cached r;
    r.YpX = q.YmX;
    r.YmX = q.YpX;
    r.Z = q.Z;
    r.T2d = fe_carry(fe_neg(q.T2d));
    return r;
}

// p + q (both projective)
NW_HD ge_p3 ge_add(const ge_p3& p, const ge_cached& q) {
    const fe a = fe_mul(fe_sub(p.Y, p.X), q.YmX);
    const fe b = fe_mul(fe_add(p.Y, p.X), q.YpX);
    const fe c = fe_mul(p.T, q.T2d);
    const fe zz = fe_mul(p.Z, q.Z);
    const fe d = fe_add(zz, zz);
    const fe e = fe_sub(b, a);
    const fe h = fe_add(b, a);
    const fe f = fe_sub(d, c);
    const fe g = fe_add(d, c);
    ge_p3 r;
    r.X = fe_mul(e, f);
    r.Y = fe_mul(g, h);
    r.Z = fe_mul(g, f);
    r.T = fe_mul(e, h);
    return r;
}

// 2p (dbl-2008-hwcd, a = -1)
NW_HD ge_p3 ge_dbl(const ge_p3& p) {
    const fe xx = fe_sq(p.X);
    const fe yy = fe_sq(p.Y);
    const fe zz = fe_sq(p.Z);
    const fe zz2 = fe_add(zz, zz);
    const fe s = fe_sq(fe_add(p.X, p.Y));
    const fe yr = fe_add(yy, xx);        // k=2
    const fe zr = fe_sub(yy, xx);        // tight
    const fe xr = fe_sub(s, yr);         // tight
    const fe tr = fe_sub(zz2, zr);       // tight
    ge_p3 r;
    r.X = fe_mul(xr, tr);
    r.Y = fe_mul(yr, zr);
    r.Z = fe_mul(zr, tr);
    r.T = fe_mul(xr, yr);
    return r;
}

NW_HD ge_p3 ge_neg(const ge_p3& p) {
    ge_p3 r = p;
    r.X = fe_carry(fe_neg(p.X));
    r.T = fe_carry(fe_neg(p.T));
    return r;
}

NW_HD ge_p3 ge_select(const ge_p3& a, const ge_p3& b, bool take_b) {
    ge_p3 r;
    r.X = fe_select(a.X, b.X, take_b);
    r.Y = fe_select(a.Y, b.Y, take_b);
    r.Z = fe_select(a.Z, b.Z, take_b);
    r.T = fe_select(a.T, b.T, take_b);
    return r;
}

// EdwardsPoint::is_identity (projective): X == 0 and Y == Z.
NW_HD bool ge_is_identity(const ge_p3& p) {
    return fe_iszero(p.X) && fe_eq(p.Y, p.Z);
}

// Projective equality (EdwardsPoint::ct_eq): X1 Z2 == X2 Z1 and Y1 Z2 == Y2 Z1.
NW_HD bool ge_eq(const ge_p3& p, const ge_p3& q) {
    return fe_eq(fe_mul(p.X, q.Z), fe_mul(q.X, p.Z)) && fe_eq(fe_mul(p.Y, q.Z), fe_mul(q.Y, p.Z));
}

// curve25519-dalek CompressedEdwardsY::decompress (oracle/ed25519_oracle.py decompress):
// y taken mod p without rejecting y >= p; sqrt_ratio_i failure -> false; x negated when the
// sign bit is set (x = 0 with the sign bit set is accepted).
NW_HD bool ge_decompress(ge_p3& out, const uint32_t w[8]) {
    const fe y = fe_frombytes_w(w);
    const fe yy = fe_sq(y);
    const fe u = fe_sub(yy, fe_one());
    const fe v = fe_add(fe_mul(yy, fe_from_const(FE_D)), fe_one());
    fe x;
    const bool ok = fe_sqrt_ratio_i(x, u, v);
    const bool sign = (w[7] >> 31) != 0;
    x = fe_select(x, fe_carry(fe_neg(x)), sign);
    out.X = x;
    out.Y = fe_carry(y);
    out.Z = fe_one();
    out.T = fe_mul(x, y);
    return ok;
}

// Canonical compressed encoding (8 LE words): y with the sign of x in bit 255.
NW_HD void ge_compress_w(uint32_t out[8], const ge_p3& p) {
    const fe zi = fe_invert_sg(p.Z);
    uint32_t xw[8];
    fe_tobytes_w(xw, fe_mul(p.X, zi));
    fe_tobytes_w(out, fe_mul(p.Y, zi));
    out[7] |= (xw[0] & 1u) << 31;
}

NW_HD bool words_eq8(const uint32_t a[8], const uint32_t b[8]) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d |= a[i] ^ b[i];
    return d == 0;
}

// A point with canonical affine y = yw is of small order (order | 8) iff y is one of the five
// y-coordinates of E[8]: 0, 1, -1, +-y8.
NW_HD bool y_is_small_order(const uint32_t yw[8]) {
    return words_eq8(yw, Y_SMALL_0) || words_eq8(yw, Y_SMALL_1) || words_eq8(yw, Y_SMALL_M1) ||
           words_eq8(yw, Y_SMALL_8) || words_eq8(yw, Y_SMALL_M8);
}

// Conditionally negate an affine Niels entry: -(x, y) = (-x, y) swaps y+x / y-x and negates 2dxy.
NW_HD ge_precomp ge_precomp_cneg(const ge_precomp& q, bool neg) {
    ge_precomp r = q;
    const uint32_t m = lane_mask(neg);
    fe_cswap_mask(r.ypx, r.ymx, m);
    r.xy2d = fe_select_mask(q.xy2d, fe_neg(q.xy2d), m);   // k <= 2
    return r;
}

NW_HD ge_precomp ge_precomp_from_words(const uint32_t* w) {
    ge_precomp q;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        q.ypx.v[i] = w[ENT_YPX + i];
        q.ymx.v[i] = w[ENT_YMX + i];
        q.xy2d.v[i] = w[ENT_XY2D + i];
    }
    return q;
}

// The 32 words of a table entry (the layout above).
NW_HD void precomp_to_words(const ge_precomp& q, uint32_t* w) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        w[ENT_YPX + i] = q.ypx.v[i];
        w[ENT_YMX + i] = q.ymx.v[i];
        w[ENT_XY2D + i] = q.xy2d.v[i];
    }
    w[10] = 0;
    w[11] = 0;
}

// Table-entry (halved affine Niels) form of p (one inversion); tight limbs.
NW_HD ge_precomp ge_to_precomp(const ge_p3& p) {
    const fe zi = fe_invert_sg(p.Z);
    return ge_precomp_from_affine(fe_mul(p.X, zi), fe_mul(p.Y, zi));
}

// Signed radix-2^W recoding, consumed one digit per call: s holds the remaining scalar bits
// (8 LE words, value < 2^253 so the top digit never carries out).  Returns d in [-2^(W-1), 2^(W-1)].
template <int W>
NW_HD int next_digit(uint32_t s[8], int& carry) {
    const int b = (int)(s[0] & ((1u << W) - 1u)) + carry;
    carry = (b + (1 << (W - 1))) >> W;
    const int d = b - (carry << W);
#pragma unroll
    for (int k = 0; k < 7; ++k) s[k] = (s[k] >> W) | (s[k + 1] << (32 - W));
    s[7] >>= W;
    return d;
}

// Variable-base k*P for a scalar of NW 32-bit LE words, binary method with a uniform add per bit
// (used only on the rare exact-batch path and at committee load).  The scalar is consumed by
// shifting, so no runtime-indexed array is needed.
template <int NW>
NW_HD ge_p3 ge_scalarmult_vartime(const uint32_t* kin, const ge_p3& p) {
    uint32_t k[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) k[i] = kin[i];
    const ge_cached pc = ge_to_cached(p);
    ge_p3 acc = ge_identity();
#pragma nounroll
    for (int i = 0; i < 32 * NW; ++i) {
        acc = ge_dbl(acc);
        const bool bit = (k[NW - 1] >> 31) != 0;
#pragma unroll
        for (int j = NW - 1; j > 0; --j) k[j] = (k[j] << 1) | (k[j - 1] >> 31);
        k[0] <<= 1;
        const ge_p3 t = ge_add(acc, pc);
        acc = ge_select(acc, t, bit);
    }
    return acc;
}

}  // namespace nw
