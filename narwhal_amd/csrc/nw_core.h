// Per-lane building blocks of the verify / sign kernels, shared with the test-only host harness
// (tools/hostcheck.hip) so the exact code the GPU runs is unit-tested against the oracle.
#pragma once
#include "nw_point.h"
#include "nw_sha512.h"
#include "nw_chacha.h"
#include "nw_kernels.h"

namespace nw {

// Ordering between the lanes of ONE wave (LDS or global data other lanes of the wave wrote):
// workgroup-scope fences (they wait for the wave's outstanding memory operations) around a
// wave-level barrier; replaces __syncthreads where the block's other waves are independent or gone.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Batch coefficient z_i of vote i of certificate ``cert`` (NW-Z v1: nonce = global certificate index).
__device__ __forceinline__ void coeff_z(const VerifyParams& a, uint32_t i, uint32_t cert, uint32_t z4[4]) {
    const uint64_t bidx = a.cert_base + cert;
    chacha20_z(z4, a.zseed, i - a.cert_first[cert], (uint32_t)bidx, (uint32_t)(bidx >> 32), 0u);
}

// ------------------------------------------------------------------------------------ loads
NW_HD void load_w8(uint32_t w[8], const uint32_t* p) {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0];
    const uint4 b = reinterpret_cast<const uint4*>(p)[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

NW_HD ge_precomp load_precomp(const uint32_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint32_t w[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 t = q[k];
        w[4 * k] = t.x; w[4 * k + 1] = t.y; w[4 * k + 2] = t.z; w[4 * k + 3] = t.w;
    }
    return ge_precomp_from_words(w);
}

NW_HD void store_p3(uint32_t* dst, const ge_p3& p) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        dst[k] = p.X.v[k];
        dst[10 + k] = p.Y.v[k];
        dst[20 + k] = p.Z.v[k];
        dst[30 + k] = p.T.v[k];
    }
}

NW_HD ge_p3 load_p3(const uint32_t* src) {
    ge_p3 p;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        p.X.v[k] = src[k];
        p.Y.v[k] = src[10 + k];
        p.Z.v[k] = src[20 + k];
        p.T.v[k] = src[30 + k];
    }
    return p;
}

__device__ __forceinline__ ge_p3 ge_shfl_down(const ge_p3& p, unsigned off) {
    ge_p3 r;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        r.X.v[k] = __shfl_down(p.X.v[k], off, 64);
        r.Y.v[k] = __shfl_down(p.Y.v[k], off, 64);
        r.Z.v[k] = __shfl_down(p.Z.v[k], off, 64);
        r.T.v[k] = __shfl_down(p.T.v[k], off, 64);
    }
    return r;
}

// Moves a wave-uniform point into VGPRs behind an optimizer barrier.  Without it the serial chains
// of k_msm_final / k_points_identity / k_cert_finalize (uniform: one batch per wave) are scalarized onto the SALU,
// which has no 32x32->64 multiply-add: PMC showed 800 k SALU vs 61 k VALU instructions per wave
// and 1.6 ms per k_msm_final launch.
__device__ __forceinline__ ge_p3 ge_to_vgpr(ge_p3 p) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        asm volatile("" : "+v"(p.X.v[k]));
        asm volatile("" : "+v"(p.Y.v[k]));
        asm volatile("" : "+v"(p.Z.v[k]));
        asm volatile("" : "+v"(p.T.v[k]));
    }
    return p;
}


// Byte of the virtual hram stream (R || A || M) at position pos >= 64, with SHA padding.
NW_HD uint32_t stream_byte(const uint8_t* msg, uint64_t len, uint64_t pos) {
    const uint64_t m = pos - 64;
    if (m < len) return msg[m];
    return m == len ? 0x80u : 0u;
}

NW_HD uint64_t stream_word(const uint8_t* msg, uint64_t len, uint64_t pos) {
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) w = (w << 8) | stream_byte(msg, len, pos + j);
    return w;
}

// SHA-512(R || A || msg[0..len)) for an arbitrary-length message.
NW_HD void hram_generic(uint32_t out[16], const uint32_t R[8], const uint32_t A[8],
                             const uint8_t* msg, uint64_t len) {
    const uint64_t total = 64 + len;
    const uint64_t nblocks = (total + 17 + 127) / 128;
    uint64_t st[8];
    sha512_init(st);
    uint64_t w[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = be64_from_le32(R[2 * k], R[2 * k + 1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[4 + k] = be64_from_le32(A[2 * k], A[2 * k + 1]);
#pragma unroll
    for (int k = 8; k < 16; ++k) w[k] = stream_word(msg, len, 8 * k);
    if (nblocks == 1) {
        w[14] = 0;
        w[15] = total * 8;
    }
    sha512_compress(st, w);
    for (uint64_t b = 1; b < nblocks; ++b) {
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = stream_word(msg, len, b * 128 + 8 * k);
        if (b == nblocks - 1) {
            w[14] = 0;
            w[15] = total * 8;
        }
        sha512_compress(st, w);
    }
    sha512_digest_le32(out, st);
}

// A table entry as gathered for a signed digit: (y-x)/2 and (y+x)/2 loaded in the order the sign
// needs (swapped for a negative digit: -q = ((y-x)/2, (y+x)/2, -d x y)), d x y as stored.
// Unpacked: each half is two 16-B loads and one 8-B load; the two pad words are never fetched.
struct ent_sw {
    uint4 m0, m1, p0, p1, c1, c2;
    uint2 m2, p2, c0;
};

NW_HD ent_sw load_ent_sw(const uint32_t* __restrict__ e, bool neg) {
    ent_sw r;
    const uint32_t* m = e + (neg ? ENT_YPX : ENT_YMX);   // pairs with Y - X
    const uint32_t* p = e + (neg ? ENT_YMX : ENT_YPX);   // pairs with Y + X
    r.m0 = reinterpret_cast<const uint4*>(m)[0];
    r.m1 = reinterpret_cast<const uint4*>(m)[1];
    r.m2 = reinterpret_cast<const uint2*>(m)[4];
    r.p0 = reinterpret_cast<const uint4*>(p)[0];
    r.p1 = reinterpret_cast<const uint4*>(p)[1];
    r.p2 = reinterpret_cast<const uint2*>(p)[4];
    r.c0 = reinterpret_cast<const uint2*>(e + ENT_XY2D)[0];
    r.c1 = reinterpret_cast<const uint4*>(e + ENT_XY2D + 2)[0];
    r.c2 = reinterpret_cast<const uint4*>(e + ENT_XY2D + 2)[1];
    return r;
}

NW_HD fe fe_from_q2(const uint4& a, const uint4& b, const uint2& c) {
    fe f;
    f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
    f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
    f.v[8] = c.x; f.v[9] = c.y;
    return f;
}

// ypx / ymx as loaded (swapped for a negative digit), xy2d as stored (its sign: ge_madd_sgn)
NW_HD ge_precomp ent_sw_precomp(const ent_sw& e) {
    ge_precomp q;
    q.ymx = fe_from_q2(e.m0, e.m1, e.m2);
    q.ypx = fe_from_q2(e.p0, e.p1, e.p2);
    fe c;
    c.v[0] = e.c0.x; c.v[1] = e.c0.y;
    c.v[2] = e.c1.x; c.v[3] = e.c1.y; c.v[4] = e.c1.z; c.v[5] = e.c1.w;
    c.v[6] = e.c2.x; c.v[7] = e.c2.y; c.v[8] = e.c2.z; c.v[9] = e.c2.w;
    q.xy2d = c;
    return q;
}

// The chain's first entry: the fully signed entry (d x y negated too) as an extended point.
NW_HD ge_p3 ent_sw_first(const ent_sw& e, bool neg) {
    ge_precomp q = ent_sw_precomp(e);
    q.xy2d = fe_select_mask(q.xy2d, fe_neg(q.xy2d), lane_mask(neg));
    return ge_from_precomp(q);
}

// One comb pass: P += sum_pos sign(d_pos) * T[pos][|d_pos|] for the signed radix-2^W digits of
// sc (consumed).  Software-pipelined: the gather of position pos+1's entry is issued before the
// mixed addition of position pos, so the (HBM) latency hides under ~1.1k VALU instructions of
// field arithmetic.  neg_pos: negate entries for positive digits (-h A).  FIRST: P is the identity
// on entry, so position 0's entry becomes P directly (ge_from_precomp: 1 multiplication, not 7).
// (Measured and rejected: two positions per iteration with two alternating buffers, to drop the
// buffer copy: it spills at the 168-VGPR bound; issuing the gather between the two halves of the
// addition (ge_madd_s1 / ge_madd_s2) to free the buffer's registers for a three-product first half:
// that still spills.)
template <int W, bool FIRST, bool FUSED = false>
NW_HD void comb_pass(ge_p3& P, uint32_t sc[8], const uint32_t* __restrict__ tab, bool neg_pos) {
    int carry = 0;
    int d = next_digit<W>(sc, carry);
    bool ng = neg_pos ? d > 0 : d < 0;
    ent_sw cur = load_ent_sw(tab + (size_t)(d < 0 ? -d : d) * PRECOMP_WORDS, ng);
    int pos = 0;
    if constexpr (FIRST) {
        // position 0 starts the chain: P = T[0][|d|] (sign applied), no addition
        const ent_sw e0 = cur;
        const bool neg0 = ng;
        d = next_digit<W>(sc, carry);   // position 1's digit; its gather overlaps the conversion
        ng = neg_pos ? d > 0 : d < 0;
        cur = load_ent_sw(tab + ((size_t)comb_ent(W) + (d < 0 ? -d : d)) * PRECOMP_WORDS, ng);
        P = ent_sw_first(e0, neg0);
        pos = 1;
    }
#pragma nounroll
    for (; pos < comb_pos(W); ++pos) {
        int dn = 0;
        bool ngn = false;
        ent_sw nxt;
        if (pos + 1 < comb_pos(W)) {
            dn = next_digit<W>(sc, carry);
            ngn = neg_pos ? dn > 0 : dn < 0;
            nxt = load_ent_sw(tab + ((size_t)(pos + 1) * comb_ent(W) + (dn < 0 ? -dn : dn)) * PRECOMP_WORDS, ngn);
        }
        P = ge_madd_sgn<FUSED>(P, ent_sw_precomp(cur), lane_mask(ng));
        cur = nxt;
        d = dn;
        ng = ngn;
    }
}

// comb_pass with the signed digits precomputed (dig[pos * stride], the lane's slot of a shared
// array): the 8-word scalar and its carry are not live during the additions (k_verify).
// NT: the table is followed by its negated copy T- (tab + comb_words(W), k_comb_negate): a digit's
// sign only picks the address, and the addition is the plain ge_madd (no swap, no f/g selects).
// LAST: the chain's final addition computes X, Y, Z only (ge_madd_s2_xyz; P.T is left zero).
template <int W, bool FIRST, bool FUSED, bool NT = false, bool LAST = false>
__device__ __forceinline__ void comb_pass_dig(ge_p3& P, const int* dig, int stride, const uint32_t* __restrict__ tab,
                                              bool neg_pos) {
    auto gather = [&](int pos, int d, bool ng) -> ent_sw {
        const uint32_t* e = tab + ((size_t)pos * comb_ent(W) + (d < 0 ? -d : d)) * PRECOMP_WORDS;
        if constexpr (NT) return load_ent_sw(e + (ng ? comb_words(W) : 0), false);
        else return load_ent_sw(e, ng);
    };
    int d = dig[0];
    bool ng = neg_pos ? d > 0 : d < 0;
    ent_sw cur = gather(0, d, ng);
    int pos = 0;
    if constexpr (FIRST) {
        const ent_sw e0 = cur;
        const bool neg0 = ng;
        d = dig[stride];
        ng = neg_pos ? d > 0 : d < 0;
        cur = gather(1, d, ng);
        if constexpr (NT) P = ge_from_precomp(ent_sw_precomp(e0));
        else P = ent_sw_first(e0, neg0);
        pos = 1;
    }
    auto add = [&](const ent_sw& e, bool n) {
        if constexpr (NT) P = ge_madd<FUSED>(P, ent_sw_precomp(e));
        else P = ge_madd_sgn<FUSED>(P, ent_sw_precomp(e), lane_mask(n));
    };
    auto sign = [&](int dd) { return neg_pos ? dd > 0 : dd < 0; };
    constexpr int END = comb_pos(W) - (LAST ? 1 : 0);   // positions [pos, END) take a full addition
#pragma nounroll
    for (; pos < END; ++pos) {
        int dn = 0;
        bool ngn = false;
        ent_sw nxt;
        if (pos + 1 < comb_pos(W)) {
            dn = dig[(pos + 1) * stride];
            ngn = sign(dn);
            nxt = gather(pos + 1, dn, ngn);
        }
        add(cur, ng);
        cur = nxt;
        d = dn;
        ng = ngn;
    }
    if constexpr (LAST) {
        if constexpr (NT) P = ge_madd_s2_xyz<FUSED>(ge_madd_s1<FUSED>(P, ent_sw_precomp(cur)));
        else P = ge_madd_s2_xyz<FUSED>(ge_madd_s1_sgn<FUSED>(P, ent_sw_precomp(cur), lane_mask(ng)));
    }
}

// P = s B - h A: radix-2^WB comb over the basepoint table, then radix-2^WA comb over the key
// table (WA = 0: s B only).  Each step is one gather + one mixed addition, no doublings.
template <int WB, int WA, bool FUSED = false>
NW_HD ge_p3 comb_sB_minus_hA(const uint32_t s_in[8], const uint32_t h_in[8], const uint32_t* __restrict__ btab,
                             const uint32_t* __restrict__ atab) {
    uint32_t s[8], h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s[k] = s_in[k];
        h[k] = h_in[k];
    }
    ge_p3 P;
    comb_pass<WB, true, FUSED>(P, s, btab, false);
    if constexpr (WA > 0) comb_pass<WA, false, FUSED>(P, h, atab, true);
    return P;
}

// h = SHA-512(R || A || M) mod l for a 32-byte message (certificate / vote digest): one block.
NW_HD void hram_msg32(uint32_t h[8], const uint32_t R[8], const uint32_t A[8], const uint32_t M[8]) {
    uint32_t m[24];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        m[k] = R[k];
        m[8 + k] = A[k];
        m[16 + k] = M[k];
    }
    uint32_t hw[16];
    sha512_oneblock_le32<24>(hw, m);
    sc_reduce512(h, hw);
}

// P = s B - h A (s forced to 0 when non-canonical so the comb's digit range stays valid).
template <int WA, int WB = B_WINDOW, bool FUSED = false>
NW_HD ge_p3 compute_P(const uint32_t S[8], const uint32_t h[8], bool sok, const uint32_t* btab,
                      const uint32_t* atab) {
    uint32_t s_use[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s_use[k] = sok ? S[k] : 0u;
    return comb_sB_minus_hA<WB, WA, FUSED>(s_use, h, btab, atab);
}

NW_HD fe load_fe(const uint32_t* p) {
    fe f;
#pragma unroll
    for (int k = 0; k < 10; ++k) f.v[k] = p[k];
    return f;
}

NW_HD void store_fe(uint32_t* p, const fe& f) {
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = f.v[k];
}

// Struct-of-arrays field element: limb k of column g at p[k * n + g].
NW_HD fe load_fe_soa(const uint32_t* p, size_t n, size_t g) {
    fe f;
#pragma unroll
    for (int k = 0; k < 10; ++k) f.v[k] = p[k * n + g];
    return f;
}

NW_HD void store_fe_soa(uint32_t* p, size_t n, size_t g, const fe& f) {
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k * n + g] = f.v[k];
}

// k_verify -> k_finish record, struct-of-arrays in processing order: X rows 0..9, Z rows 10..19,
// partial flags row 20 (PREC_ROWS rows of n words).
static constexpr int PREC_ROWS = 21;
static constexpr int PREC_FLAGS_ROW = 20;
static_assert(PREC_ROWS <= PBUF_WORDS, "pbuf workspace rows");
static constexpr uint32_t PF_YMATCH = 1u << 20;   // internal: y_R Z == Y (projective)
static constexpr uint32_t PF_RSIGN = 1u << 21;    // internal: R's sign bit (bit 255)
static constexpr uint32_t PF_NOCERT = 1u << 22;   // internal: the signature is in no certificate's range
static constexpr uint32_t PF_INTERNAL = PF_YMATCH | PF_RSIGN | PF_NOCERT;

NW_HD void store_prec_soa(uint32_t* p, size_t n, size_t g, const ge_p3& P, uint32_t pflags) {
    store_fe_soa(p, n, g, P.X);
    store_fe_soa(p + 10 * n, n, g, P.Z);
    p[PREC_FLAGS_ROW * n + g] = pflags;
}

// The half of the encoding match that needs no inversion (run in k_verify, where P is live):
//   y:  decode(R).y == P.y  <=>  y_R Z == Y  (y_R = R's y field as FieldElement::from_bytes reads
//       it, i.e. taken mod p); when it holds, R decodes (P.x^2 is the ratio sqrt_ratio_i roots)
//   R small order (meaningful when MATCH): canonical y_R is one of the five y's of E[8]
//   R's sign bit, for k_finish's parity check.
NW_HD uint32_t verify_pflags(const ge_p3& P, const uint32_t R[8], uint32_t partial) {
    const fe yR = fe_frombytes_w(R);
    const bool ymatch = fe_iszero(fe_sub(fe_mul(yR, P.Z), P.Y));
    uint32_t yr[8];
    fe_tobytes_w(yr, yR);
    return partial | (ymatch ? PF_YMATCH : 0u) | ((R[7] >> 31) ? PF_RSIGN : 0u) |
           (y_is_small_order(yr) ? NW_F_R_SMALL : 0u);
}

// The other half, after the batch inversion (zi = 1/Z): x = X zi; decode(R) == P iff the y's match
// and x = 0 or x's parity is R's sign bit (dalek's decompress negates the non-negative root when
// the sign bit is set, and accepts x = 0 with the sign bit set).
//   MATCH  <=> R decodes (dalek decompress) and decode(R) == P  (the strict equation R = sB - hA)
//   STRICT <=> verify_strict accepts (adds: S ok, A ok, neither R nor A of small order)
NW_HD uint32_t finish_flags(uint32_t pf, bool xmatch) {
    const bool match = (pf & PF_YMATCH) && xmatch;
    const bool sok = (pf & NW_F_S_OK) != 0, aok = (pf & NW_F_A_OK) != 0;
    const bool asmall = (pf & NW_F_A_SMALL) != 0, rsmall = (pf & NW_F_R_SMALL) != 0;
    const bool strict = sok && aok && match && !asmall && !rsmall;
    return (pf & ~PF_INTERNAL) | (match ? NW_F_MATCH : 0u) | (strict ? NW_F_STRICT : 0u);
}

NW_HD uint32_t finish_x_flags(const fe& X, const fe& zi, uint32_t pf) {
    uint32_t xw[8];
    fe_tobytes_w(xw, fe_mul(X, zi));
    const bool x_zero = (xw[0] | xw[1] | xw[2] | xw[3] | xw[4] | xw[5] | xw[6] | xw[7]) == 0;
    return finish_flags(pf, x_zero || ((xw[0] & 1u) == ((pf & PF_RSIGN) ? 1u : 0u)));
}

// A signature's final flags f (pf: its partial flags) stored, with the exact-path bookkeeping of a
// batch call: a vote in no certificate's range gets no verdict; a parse / decode failure dooms its
// certificate (dalek errors before the MSM); a mismatch joins the exact-path list.  k_finish, and
// k_verify_split when it does k_finish's work itself (small launches).
__device__ __forceinline__ void finish_emit(const VerifyParams& a, uint32_t i, uint32_t pf, uint32_t f) {
    if (a.batch_mode) {
        if (pf & PF_NOCERT) {
            f = 0u;
        } else if ((f & (NW_F_S_OK | NW_F_A_OK)) != (NW_F_S_OK | NW_F_A_OK)) {
            atomicOr(&a.cert_state[a.sig_cert[i]], CS_DOOM);
        } else if (!(f & NW_F_MATCH)) {
            f |= NW_F_SLOW;
            const uint32_t t = atomicAdd(a.slow_count, 1u);
            a.slow_list[t] = i;
            a.slow_slot[i] = t;
        }
    }
    a.flags[i] = f;
    if (a.ok_out) a.ok_out[i] = (f & NW_F_STRICT) ? 1 : 0;
}

// Flags from P (with zi = 1/Z_P) against the signature's R encoding (both halves).
NW_HD uint32_t match_flags(const ge_p3& P, const fe& zi, const uint32_t R[8], bool sok, bool aok, bool asmall) {
    const uint32_t partial = (sok ? NW_F_S_OK : 0u) | (aok ? NW_F_A_OK : 0u) | (asmall ? NW_F_A_SMALL : 0u);
    return finish_x_flags(P.X, zi, verify_pflags(P, R, partial));
}

// Torsion coefficient of signature i: ((r - z h) mod 8) * t mod 8 with r = z h mod l
// (the -5 q_i A_i^t term of the exact batch decomposition; A_i^t = t T8).
NW_HD uint32_t torsion_coef(const uint32_t z4[4], const uint32_t h[8], uint32_t t) {
    uint32_t z8[8] = {z4[0], z4[1], z4[2], z4[3], 0u, 0u, 0u, 0u};
    uint32_t r[8];
    sc_mul(r, z8, h);
    const uint32_t zh0 = (z4[0] * h[0]) & 7u;
    return (((r[0] - zh0) & 7u) * t) & 7u;
}

// Q_i = z_i (R_i - P_i) for a signature whose strict equation fails.
NW_HD ge_p3 slow_term(const ge_p3& Rp, const ge_p3& P, const uint32_t z4[4]) {
    const ge_p3 D = ge_add(Rp, ge_cached_neg(ge_to_cached(P)));
    return ge_scalarmult_vartime<4>(z4, D);
}

// Generator T8 of the (cyclic) 8-torsion subgroup E[8].
NW_HD ge_p3 ge_t8() {
    ge_p3 T8;
    T8.X = fe_from_const(FE_T8X);
    T8.Y = fe_from_const(FE_T8Y);
    T8.Z = fe_one();
    T8.T = fe_mul(T8.X, T8.Y);
    return T8;
}

// Key cache preparation for one key: returns key_info bits and writes the comb bases
// 2^(W pos) * A (extended, 40 words each).  Undecodable keys use the identity (their verdicts are
// Err regardless) so every table entry stays a valid curve point.
template <int W>
NW_HD uint32_t key_prep_one(const uint32_t* raw, uint32_t* bases) {
    uint32_t w[8];
    load_w8(w, raw);
    ge_p3 A;
    const bool ok = ge_decompress(A, w);
    if (!ok) A = ge_identity();
    const ge_p3 A8 = ge_dbl(ge_dbl(ge_dbl(A)));
    const bool small = ge_is_identity(A8);
    const ge_p3 At = ge_scalarmult_vartime<8>(SC_5L, A);
    const ge_cached t8c = ge_to_cached(ge_t8());
    ge_p3 Q = ge_identity();
    uint32_t t = 0;
    for (uint32_t k = 0; k < 8; ++k) {
        if (ge_eq(Q, At)) t = k;
        Q = ge_add(Q, t8c);
    }
    ge_p3 cur = A;
    for (int pos = 0; pos < comb_pos(W); ++pos) {
        store_p3(bases + (size_t)pos * 40, cur);
        for (int d = 0; d < W; ++d) cur = ge_dbl(cur);
    }
    return (ok ? KI_OK : 0u) | (small ? KI_SMALL : 0u) | (t << KI_TORSION_SHIFT);
}

// Comb entry e (0..2^(W-1)) of position pos: e * 2^(W pos) * A in affine Niels form.
template <int W>
NW_HD void comb_entry_one(const uint32_t* bases, uint32_t pos, uint32_t e, uint32_t* tab) {
    ge_precomp q;
    if (e == 0) {
        q = ge_precomp_identity();
    } else {
        const ge_p3 base = load_p3(bases + (size_t)pos * 40);
        const ge_cached bc = ge_to_cached(base);
        ge_p3 acc = ge_identity();
        for (int b = W - 1; b >= 0; --b) {
            acc = ge_dbl(acc);
            if ((e >> b) & 1u) acc = ge_add(acc, bc);
        }
        q = ge_to_precomp(acc);
    }
    uint32_t* dst = tab + ((size_t)pos * comb_ent(W) + e) * PRECOMP_WORDS;
    uint32_t w[32];
    precomp_to_words(q, w);
#pragma unroll
    for (int k = 0; k < 32; ++k) dst[k] = w[k];
}

// Comb-table builder for entries [CH c, CH c + CH) of one (key, position): consecutive multiples
// Q_k = (CH c + k) * base by repeated addition, then ONE field inversion for the whole chunk
// (Montgomery's trick, prefix products kept in registers) to reach affine Niels form.  The chunk's
// projective X, Y, Z are parked in their own table slots between the two passes.  About 90 field
// multiplications per entry instead of ~500 for a per-entry double-and-add plus inversion.
template <int W, int CH>
NW_HD void comb_chunk_build(const uint32_t* bases, uint32_t pos, uint32_t c, uint32_t* tab) {
    constexpr uint32_t ENT = (uint32_t)comb_ent(W);
    constexpr int NB = 32 - __builtin_clz((ENT - 1) / CH);   // bits of the largest chunk index
    const uint32_t e0 = c * CH;
    const uint32_t cnt = ENT - e0 < (uint32_t)CH ? ENT - e0 : (uint32_t)CH;
    const ge_p3 base = load_p3(bases + (size_t)pos * 40);
    const ge_cached bc = ge_to_cached(base);
    ge_p3 stride = base;
#pragma unroll
    for (int k = 1; k < CH; k <<= 1) stride = ge_dbl(stride);
    const ge_cached sc = ge_to_cached(stride);
    ge_p3 Q = ge_identity();   // Q = c * stride, uniform double-and-add over NB bits
#pragma nounroll
    for (int b = NB - 1; b >= 0; --b) {
        Q = ge_dbl(Q);
        const ge_p3 Qa = ge_add(Q, sc);
        Q = ge_select(Q, Qa, ((c >> b) & 1u) != 0);
    }
    uint32_t* slot0 = tab + ((size_t)pos * ENT + e0) * PRECOMP_WORDS;
    fe pre[CH];
    fe acc = fe_one();
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        if ((uint32_t)k < cnt) {
            uint32_t* sl = slot0 + (size_t)k * PRECOMP_WORDS;
            store_fe(sl, Q.X);
            store_fe(sl + 10, Q.Y);
            store_fe(sl + 20, Q.Z);
            acc = fe_mul(acc, Q.Z);
            pre[k] = acc;
            if ((uint32_t)k + 1 < cnt) Q = ge_add(Q, bc);
        }
    }
    fe inv = fe_invert_sg(acc);
#pragma unroll
    for (int k = CH - 1; k >= 0; --k) {
        if ((uint32_t)k < cnt) {
            uint32_t* sl = slot0 + (size_t)k * PRECOMP_WORDS;
            const fe Z = load_fe(sl + 20);
            fe zi = inv;
            if (k > 0) {
                zi = fe_mul(inv, pre[k - 1]);
                inv = fe_mul(inv, Z);
            }
            const fe x = fe_mul(load_fe(sl), zi);
            const fe y = fe_mul(load_fe(sl + 10), zi);
            const ge_precomp q = ge_precomp_from_affine(x, y);
            uint32_t w[32];
            precomp_to_words(q, w);
#pragma unroll
            for (int j = 0; j < 32; ++j) sl[j] = w[j];
        }
    }
}

// RFC 8032 Ed25519 signing of an MW-word message (crypto::Signature::new, crypto/src/lib.rs:185-191).
template <int MW, int WB = B_WINDOW>
NW_HD void sign_one(const uint32_t* seed_in, const uint32_t* msg_in, const uint32_t* btab, uint32_t pk[8],
                    uint32_t sig[16]) {
    uint32_t seed[8], m[MW];
#pragma unroll
    for (int k = 0; k < 8; ++k) seed[k] = seed_in[k];
#pragma unroll
    for (int k = 0; k < MW; ++k) m[k] = msg_in[k];
    uint32_t hs[16];
    sha512_oneblock_le32<8>(hs, seed);
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = hs[k];
    a[0] &= 0xFFFFFFF8u;
    a[7] &= 0x7FFFFFFFu;
    a[7] |= 0x40000000u;
    uint32_t wide[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) wide[k] = k < 8 ? a[k] : 0u;
    uint32_t ared[8];
    sc_reduce512(ared, wide);
    uint32_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t Aw[8];
    ge_compress_w(Aw, comb_sB_minus_hA<WB, 0>(ared, zero8, btab, nullptr));
    uint32_t pm[8 + MW];
#pragma unroll
    for (int k = 0; k < 8; ++k) pm[k] = hs[8 + k];
#pragma unroll
    for (int k = 0; k < MW; ++k) pm[8 + k] = m[k];
    uint32_t rh[16];
    sha512_oneblock_le32<8 + MW>(rh, pm);
    uint32_t r[8];
    sc_reduce512(r, rh);
    uint32_t Rw[8];
    ge_compress_w(Rw, comb_sB_minus_hA<WB, 0>(r, zero8, btab, nullptr));
    uint32_t ram[16 + MW];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        ram[k] = Rw[k];
        ram[8 + k] = Aw[k];
    }
#pragma unroll
    for (int k = 0; k < MW; ++k) ram[16 + k] = m[k];
    uint32_t kh[16];
    sha512_oneblock_le32<16 + MW>(kh, ram);
    uint32_t kk[8];
    sc_reduce512(kk, kh);
    uint32_t s[8];
    sc_muladd(s, kk, a, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        pk[k] = Aw[k];
        sig[k] = Rw[k];
        sig[8 + k] = s[k];
    }
}

}  // namespace nw
