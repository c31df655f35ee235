// Field inversion in GF(2^255 - 19) by Bernstein-Yang "safegcd" divsteps (constant iteration count,
// branch-free, so every lane of a wave runs the same instruction stream).
//
// Why: the Fermat chain (fe_invert: 254 squarings + 11 multiplications) is one long dependent
// sequence of ~95k VALU cycles per lane; k_finish pays one inversion per chain of FINISH_K
// signatures, and a single-certificate submission pays it on its critical path.  safegcd replaces
// it with 20 batches of 30 divsteps on the low 32 bits (plain 32-bit ops) plus, per batch, one
// 2x2 transition-matrix application to (f, g) and to the Bezout pair (d, e) (signed 32x32->64
// multiply-accumulates over nine 30-bit limbs).
//
// Algorithm (Bernstein & Yang, "Fast constant-time gcd computation and modular inversion", 2019,
// with the delta = 1/2 start and the 590-divstep bound for 256-bit moduli): f = p, g = x, d = 0,
// e = 1; each divstep maps (delta, f, g) to (1 - delta, g, (g - f)/2) when delta > 0 and g is
// odd, else to (1 + delta, f, (g + (g mod 2) f)/2), with (d, e) tracking f = d x, g = e x (mod p)
// scaled by 2^-steps.  After 600 divsteps g = 0 and f = +-1, so x^-1 = +-d.  Here zeta = -(delta
// + 1/2) so the "delta > 0" test is a sign test.
//
// Signed-30 limbs: value = sum v[i] 2^(30 i), nine limbs (270 bits), limbs in (-2^30, 2^30)
// except the top one, which carries the sign.
#pragma once
#include <cstdint>
#include "nw_field.h"

namespace nw {

struct s30 {
    int32_t v[9];
};

static constexpr int32_t S30_M = 0x3FFFFFFF;
// p = 2^255 - 19 in signed-30 limbs, and p^-1 mod 2^30.
static constexpr int32_t S30_P[9] = {0x3FFFFFED, 0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF,
                                     0x3FFFFFFF, 0x3FFFFFFF, 0x3FFFFFFF, 0x7FFF};
static constexpr uint32_t S30_PINV = 0x179435E5u;

struct s30_trans {
    int32_t u, v, q, r;
};

// 30 divsteps on the low 32 bits of f (odd) and g.  Returns the new zeta; t maps (f, g) to
// 2^30 (f', g').  Matrix entries stay in [-2^30, 2^30]; kept unsigned so the shifts are defined.
NW_HD int32_t s30_divsteps(int32_t zeta, uint32_t f, uint32_t g, s30_trans& t) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
    for (int i = 0; i < 30; ++i) {
        const uint32_t c1 = (uint32_t)(zeta >> 31);   // all-ones iff zeta < 0 (delta > 0)
        const uint32_t c2 = 0u - (g & 1u);            // all-ones iff g odd
        const uint32_t x = (f ^ c1) - c1;             // -f, -u, -v when delta > 0
        const uint32_t y = (u ^ c1) - c1;
        const uint32_t z = (v ^ c1) - c1;
        g += x & c2;
        q += y & c2;
        r += z & c2;
        const uint32_t c3 = c1 & c2;                  // swap case
        zeta = (int32_t)(((uint32_t)zeta ^ c3) - 1u);
        f += g & c3;
        u += q & c3;
        v += r & c3;
        g >>= 1;
        u += u;
        v += v;
    }
    t.u = (int32_t)u;
    t.v = (int32_t)v;
    t.q = (int32_t)q;
    t.r = (int32_t)r;
    return zeta;
}

// (f, g) <- t (f, g) / 2^30 (exact: the low 30 bits of both products are zero by construction).
NW_HD void s30_update_fg(s30& f, s30& g, const s30_trans& t) {
    int64_t cf = (int64_t)t.u * f.v[0] + (int64_t)t.v * g.v[0];
    int64_t cg = (int64_t)t.q * f.v[0] + (int64_t)t.r * g.v[0];
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        const int32_t fi = f.v[i], gi = g.v[i];
        cf += (int64_t)t.u * fi + (int64_t)t.v * gi;
        cg += (int64_t)t.q * fi + (int64_t)t.r * gi;
        f.v[i - 1] = (int32_t)cf & S30_M;
        g.v[i - 1] = (int32_t)cg & S30_M;
        cf >>= 30;
        cg >>= 30;
    }
    f.v[8] = (int32_t)cf;
    g.v[8] = (int32_t)cg;
}

// (d, e) <- (t (d, e) + p (md, me)) / 2^30 with md, me chosen so the division is exact; keeps
// d, e in (-2p, p) given they start there.
NW_HD void s30_update_de(s30& d, s30& e, const s30_trans& t) {
    const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
    int32_t md = (t.u & sd) + (t.v & se);
    int32_t me = (t.q & sd) + (t.r & se);
    int64_t cd = (int64_t)t.u * d.v[0] + (int64_t)t.v * e.v[0];
    int64_t ce = (int64_t)t.q * d.v[0] + (int64_t)t.r * e.v[0];
    md -= (int32_t)((S30_PINV * (uint32_t)cd + (uint32_t)md) & (uint32_t)S30_M);
    me -= (int32_t)((S30_PINV * (uint32_t)ce + (uint32_t)me) & (uint32_t)S30_M);
    cd += (int64_t)S30_P[0] * md;
    ce += (int64_t)S30_P[0] * me;
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < 9; ++i) {
        const int32_t di = d.v[i], ei = e.v[i];
        cd += (int64_t)t.u * di + (int64_t)t.v * ei + (int64_t)S30_P[i] * md;
        ce += (int64_t)t.q * di + (int64_t)t.r * ei + (int64_t)S30_P[i] * me;
        d.v[i - 1] = (int32_t)cd & S30_M;
        e.v[i - 1] = (int32_t)ce & S30_M;
        cd >>= 30;
        ce >>= 30;
    }
    d.v[8] = (int32_t)cd;
    e.v[8] = (int32_t)ce;
}

// r in (-2p, p) -> r * sign(sgn) mod p in [0, p), limbs in [0, 2^30).
NW_HD void s30_normalize(s30& r, int32_t sgn) {
    int32_t m = r.v[8] >> 31;   // add p if negative
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] += S30_P[i] & m;
    const int32_t n = sgn >> 31;   // negate if f ended at -1
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] = (r.v[i] ^ n) - n;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        r.v[i + 1] += r.v[i] >> 30;
        r.v[i] &= S30_M;
    }
    m = r.v[8] >> 31;
#pragma unroll
    for (int i = 0; i < 9; ++i) r.v[i] += S30_P[i] & m;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        r.v[i + 1] += r.v[i] >> 30;
        r.v[i] &= S30_M;
    }
}

// Variable-time divsteps (Bernstein-Yang as restated in Wuille's "safegcd implementation" notes,
// with eta = -delta, delta starting at 1): runs of zeros in g are consumed at once, and each odd
// g is combined with f using a multiplier w that clears min(eta + 1, remaining, 4 or 6) low bits.
// The inputs are public (verification), so variable time is acceptable; the lanes of a wave
// diverge in the iteration count, which costs the maximum over the wave, still well below the 30
// fixed branch-free steps.  Same transition-matrix contract as s30_divsteps.
NW_HD int32_t s30_divsteps_var(int32_t eta, uint32_t f, uint32_t g, s30_trans& t) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
    int i = 30;
    for (;;) {
        // sentinel bit at position i: count zeros only up to the remaining steps
        const int zeros = __builtin_ctz(g | (0xFFFFFFFFu << i));
        g >>= zeros;
        u <<= zeros;
        v <<= zeros;
        eta -= zeros;
        i -= zeros;
        if (i == 0) break;
        uint32_t w, m;
        int limit;
        if (eta < 0) {
            eta = -eta;
            uint32_t tmp = f;
            f = g;
            g = 0u - tmp;
            tmp = u;
            u = q;
            q = 0u - tmp;
            tmp = v;
            v = r;
            r = 0u - tmp;
            limit = (eta + 1) > i ? i : (eta + 1);
            m = (0xFFFFFFFFu >> (32 - limit)) & 63u;
            w = (f * g * (f * f - 2u)) & m;   // -g / f mod 2^6
        } else {
            limit = (eta + 1) > i ? i : (eta + 1);
            m = (0xFFFFFFFFu >> (32 - limit)) & 15u;
            w = f + (((f + 1u) & 4u) << 1);   // f^-1 mod 2^4
            w = (0u - w * g) & m;
        }
        g += f * w;
        q += u * w;
        r += v * w;
    }
    t.u = (int32_t)u;
    t.v = (int32_t)v;
    t.q = (int32_t)q;
    t.r = (int32_t)r;
    return eta;
}

NW_HD bool s30_is_zero(const s30& a) {
    int32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) o |= a.v[i];
    return o == 0;
}

NW_HD void fe_to_s30(s30& g, const fe& z) {
    uint32_t w[8];
    fe_tobytes_w(w, z);
    g.v[0] = (int32_t)(w[0] & S30_M);
    g.v[1] = (int32_t)(((w[0] >> 30) | (w[1] << 2)) & S30_M);
    g.v[2] = (int32_t)(((w[1] >> 28) | (w[2] << 4)) & S30_M);
    g.v[3] = (int32_t)(((w[2] >> 26) | (w[3] << 6)) & S30_M);
    g.v[4] = (int32_t)(((w[3] >> 24) | (w[4] << 8)) & S30_M);
    g.v[5] = (int32_t)(((w[4] >> 22) | (w[5] << 10)) & S30_M);
    g.v[6] = (int32_t)(((w[5] >> 20) | (w[6] << 12)) & S30_M);
    g.v[7] = (int32_t)(((w[6] >> 18) | (w[7] << 14)) & S30_M);
    g.v[8] = (int32_t)(w[7] >> 16);
}

// [0, p) in 30-bit limbs -> radix 2^25.5
NW_HD fe s30_to_fe(const s30& d) {
    uint32_t w[8];
    w[0] = (uint32_t)d.v[0] | ((uint32_t)d.v[1] << 30);
    w[1] = ((uint32_t)d.v[1] >> 2) | ((uint32_t)d.v[2] << 28);
    w[2] = ((uint32_t)d.v[2] >> 4) | ((uint32_t)d.v[3] << 26);
    w[3] = ((uint32_t)d.v[3] >> 6) | ((uint32_t)d.v[4] << 24);
    w[4] = ((uint32_t)d.v[4] >> 8) | ((uint32_t)d.v[5] << 22);
    w[5] = ((uint32_t)d.v[5] >> 10) | ((uint32_t)d.v[6] << 20);
    w[6] = ((uint32_t)d.v[6] >> 12) | ((uint32_t)d.v[7] << 18);
    w[7] = ((uint32_t)d.v[7] >> 14) | ((uint32_t)d.v[8] << 16);
    return fe_frombytes_w(w);
}

// z^-1 mod p (0 -> 0) in variable time: batches of 30 variable-time divsteps until g = 0 (for
// every lane of the wave: the loop condition is per lane, finished lanes idle).
NW_HD fe fe_invert_var(const fe& z) {
    s30 f, g, d, e;
    fe_to_s30(g, z);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        f.v[i] = S30_P[i];
        d.v[i] = 0;
        e.v[i] = 0;
    }
    e.v[0] = 1;
    int32_t eta = -1;
#pragma nounroll
    for (int it = 0; it < 40 && !s30_is_zero(g); ++it) {
        s30_trans t;
        eta = s30_divsteps_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        s30_update_de(d, e, t);
        s30_update_fg(f, g, t);
    }
    s30_normalize(d, f.v[8]);
    return s30_to_fe(d);
}

#if defined(__HIPCC__)
// ---- one inversion per wave, on the scalar unit ------------------------------------------------
// A lone lane's inversion is a serial chain of ~14 k VALU instructions that a wave issues at ~6-7
// cycles each when nothing hides the latency (k_finish's one wave per SIMD, a single header check).
// The same safegcd on WAVE-UNIFORM operands compiles to scalar (SALU) code, whose dependent
// instructions issue back to back: z is taken from the first active lane (readfirstlane) and every
// operation below is on uniform values.  Callers batch their lanes' values into one uniform product
// first (fe_invert_batched).
__device__ __forceinline__ fe fe_invert_wave(const fe& z_in) {
    fe z;
#pragma unroll
    for (int k = 0; k < 10; ++k) z.v[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)z_in.v[k]);
    return fe_invert_var(z);
}

__device__ __forceinline__ fe fe_shfl_xor(const fe& x, int off) {
    fe r;
#pragma unroll
    for (int k = 0; k < 10; ++k) r.v[k] = (uint32_t)__shfl_xor((int)x.v[k], off, 64);
    return r;
}

// z^-1 for every lane of the wave, where lanes [g*GS, g*GS + GS) all hold the same z (GS lanes per
// value; every lane of the wave active): Montgomery's trick over the wave's 64 / GS values by an
// xor butterfly (log2(64 / GS) levels of two products: the running product, identical in every lane
// at the end since each level multiplies the same pair in both partners, and the product of the
// OTHER values), one scalar-unit inversion of the wave's product, one product back.  A zero z
// contributes 1 and gets 0 (as fe_invert_var(0)).
template <int GS>
__device__ __forceinline__ fe fe_invert_batched(const fe& z) {
    const bool zz = fe_iszero(z);
    fe t = fe_select(z, fe_one(), zz);
    fe others = fe_one();
#pragma unroll
    for (int off = GS; off < 64; off <<= 1) {
        const fe p = fe_shfl_xor(t, off);
        others = fe_mul(others, p);
        t = fe_mul(t, p);
    }
    const fe r = fe_mul(fe_invert_wave(t), others);
    return fe_select(r, fe_zero(), zz);
}

// z^-1 for every lane of a workgroup of NWAVES full waves (every thread of the block calls it, one
// value per lane; 2 <= NWAVES <= 64, a power of two): the wave butterfly as above, then the NWAVES
// wave products meet in LDS, where wave 0 runs the same butterfly over them (lane w holds wave w's
// product), the block's ONE scalar-unit inversion, and hands every wave the inverse of its own
// product.  slot: __shared__ scratch of NWAVES x 10 words.  A CU's waves share one scalar unit, so
// with several waves per SIMD this cuts its work NWAVES-fold.
template <int NWAVES>
__device__ __forceinline__ fe fe_invert_block(const fe& z, uint32_t (*slot)[10]) {
    static_assert(NWAVES >= 2 && NWAVES <= 64 && (NWAVES & (NWAVES - 1)) == 0, "NWAVES: a power of two");
    const bool zz = fe_iszero(z);
    fe t = fe_select(z, fe_one(), zz);
    fe others = fe_one();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const fe p = fe_shfl_xor(t, off);
        others = fe_mul(others, p);
        t = fe_mul(t, p);
    }
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 10; ++k) slot[w][k] = t.v[k];
    }
    __syncthreads();
    if (w == 0) {
        // lanes [0, NWAVES) hold the wave products; the xor levels below NWAVES keep every group of
        // NWAVES lanes to itself, so lanes past NWAVES (ones) never reach group 0
        fe v = fe_one();
        if (lane < (uint32_t)NWAVES) {
#pragma unroll
            for (int k = 0; k < 10; ++k) v.v[k] = slot[lane][k];
        }
        fe vo = fe_one();
#pragma unroll
        for (int off = 1; off < NWAVES; off <<= 1) {
            const fe p = fe_shfl_xor(v, off);
            vo = fe_mul(vo, p);
            v = fe_mul(v, p);
        }
        const fe r = fe_mul(fe_invert_wave(v), vo);   // lane w < NWAVES: (wave w's product)^-1
        if (lane < (uint32_t)NWAVES) {
#pragma unroll
            for (int k = 0; k < 10; ++k) slot[lane][k] = r.v[k];
        }
    }
    __syncthreads();
    fe tw;
#pragma unroll
    for (int k = 0; k < 10; ++k) tw.v[k] = slot[w][k];
    const fe r = fe_mul(tw, others);
    return fe_select(r, fe_zero(), zz);
}
#endif

// z^-1 mod p (0 -> 0), same result as fe_invert.
NW_HD fe fe_invert_sg(const fe& z) {
    uint32_t w[8];
    fe_tobytes_w(w, z);
    s30 g;
    g.v[0] = (int32_t)(w[0] & S30_M);
    g.v[1] = (int32_t)(((w[0] >> 30) | (w[1] << 2)) & S30_M);
    g.v[2] = (int32_t)(((w[1] >> 28) | (w[2] << 4)) & S30_M);
    g.v[3] = (int32_t)(((w[2] >> 26) | (w[3] << 6)) & S30_M);
    g.v[4] = (int32_t)(((w[3] >> 24) | (w[4] << 8)) & S30_M);
    g.v[5] = (int32_t)(((w[4] >> 22) | (w[5] << 10)) & S30_M);
    g.v[6] = (int32_t)(((w[5] >> 20) | (w[6] << 12)) & S30_M);
    g.v[7] = (int32_t)(((w[6] >> 18) | (w[7] << 14)) & S30_M);
    g.v[8] = (int32_t)(w[7] >> 16);
    s30 f, d, e;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        f.v[i] = S30_P[i];
        d.v[i] = 0;
        e.v[i] = 0;
    }
    e.v[0] = 1;
    int32_t zeta = -1;
#pragma nounroll
    for (int it = 0; it < 20; ++it) {
        s30_trans t;
        zeta = s30_divsteps(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        s30_update_de(d, e, t);
        s30_update_fg(f, g, t);
    }
    s30_normalize(d, f.v[8]);
    // [0, p) in 30-bit limbs -> 8 LE words -> radix 2^25.5
    w[0] = (uint32_t)d.v[0] | ((uint32_t)d.v[1] << 30);
    w[1] = ((uint32_t)d.v[1] >> 2) | ((uint32_t)d.v[2] << 28);
    w[2] = ((uint32_t)d.v[2] >> 4) | ((uint32_t)d.v[3] << 26);
    w[3] = ((uint32_t)d.v[3] >> 6) | ((uint32_t)d.v[4] << 24);
    w[4] = ((uint32_t)d.v[4] >> 8) | ((uint32_t)d.v[5] << 22);
    w[5] = ((uint32_t)d.v[5] >> 10) | ((uint32_t)d.v[6] << 20);
    w[6] = ((uint32_t)d.v[6] >> 12) | ((uint32_t)d.v[7] << 18);
    w[7] = ((uint32_t)d.v[7] >> 14) | ((uint32_t)d.v[8] << 16);
    return fe_frombytes_w(w);
}

}  // namespace nw
