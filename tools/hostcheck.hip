// Test-only host harness: compiles the SAME __host__ __device__ per-lane functions the gfx950
// kernels run (nw_field/nw_scalar/nw_point/nw_sha512/nw_core) for the x86 host, so the math can
// be checked against the Python oracle in this GPU-less container (tools/hostcheck.py).
// Never linked into libnwcrypto.so; never used as a fallback.
#include <hip/hip_runtime.h>
#include <cstring>
#include <vector>
#include "../narwhal_amd/csrc/nw_core.h"
#include "../narwhal_amd/csrc/nw_inv.h"

using namespace nw;

static void b2w(uint32_t w[8], const uint8_t* b) { std::memcpy(w, b, 32); }
static void w2b(uint8_t* b, const uint32_t w[8]) { std::memcpy(b, w, 32); }

static fe fe_in(const uint8_t* b) {
    uint32_t w[8];
    b2w(w, b);
    return fe_frombytes_w(w);
}
static void fe_out(uint8_t* b, const fe& f) {
    uint32_t w[8];
    fe_tobytes_w(w, f);
    w2b(b, w);
}

template <int W>
static uint32_t build_comb_w(const uint32_t raw[8], uint32_t* bases, uint32_t* tab) {
    const uint32_t info = key_prep_one<W>(raw, bases);
    for (uint32_t pos = 0; pos < (uint32_t)comb_pos(W); ++pos)
        for (uint32_t c = 0; c < (uint32_t)(comb_ent(W) + 7) / 8; ++c) comb_chunk_build<W, 8>(bases, pos, c, tab);
    return info;
}

template <int W>
static ge_p3 compute_P_w(int w, const uint32_t S[8], const uint32_t h[8], bool sok, const uint32_t* btab,
                         const uint32_t* atab) {
    (void)w;
    return compute_P<W, 16>(S, h, sok, btab, atab);   // host harness: basepoint comb at w16
}

extern "C" {

void hc_fe_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { fe_out(out, fe_mul(fe_in(a), fe_in(b))); }
void hc_fe_sq(const uint8_t* a, uint8_t* out) { fe_out(out, fe_sq(fe_in(a))); }
void hc_fe_invert(const uint8_t* a, uint8_t* out) { fe_out(out, fe_invert(fe_in(a))); }
void hc_fe_invert_sg(const uint8_t* a, uint8_t* out) { fe_out(out, fe_invert_sg(fe_in(a))); }
void hc_fe_invert_var(const uint8_t* a, uint8_t* out) { fe_out(out, fe_invert_var(fe_in(a))); }
void hc_fe_add_sub(const uint8_t* a, const uint8_t* b, uint8_t* sum, uint8_t* diff) {
    const fe fa = fe_in(a), fb = fe_in(b);
    fe_out(sum, fe_add(fa, fb));
    fe_out(diff, fe_sub(fa, fb));
}
// stress: limbs forced to their maximum loose values (k = 2 / 3) through mul
void hc_fe_mul_loose(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out) {
    const fe fa = fe_in(a), fb = fe_in(b), fc = fe_in(c);
    const fe g = fe_add(fe_add(fa, fb), fc);   // k = 3
    const fe f = fe_add(fa, fb);               // k = 2
    fe_out(out, fe_mul(g, f));
}
void hc_fe_pow22523(const uint8_t* a, uint8_t* out) { fe_out(out, fe_pow22523(fe_in(a))); }

void hc_sc_reduce512(const uint8_t* in64, uint8_t* out) {
    uint32_t x[16], r[8];
    std::memcpy(x, in64, 64);
    sc_reduce512(r, x);
    w2b(out, r);
}
void hc_sc_muladd(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out) {
    uint32_t x[8], y[8], z[8], r[8];
    b2w(x, a);
    b2w(y, b);
    b2w(z, c);
    sc_muladd(r, x, y, z);
    w2b(out, r);
}
int hc_sc_is_canonical(const uint8_t* s) {
    uint32_t w[8];
    b2w(w, s);
    return sc_is_canonical(w) ? 1 : 0;
}

void hc_sha512_oneblock96(const uint8_t* in96, uint8_t* out64) {
    uint32_t m[24], d[16];
    std::memcpy(m, in96, 96);
    sha512_oneblock_le32<24>(d, m);
    std::memcpy(out64, d, 64);
}
void hc_hram_generic(const uint8_t* R, const uint8_t* A, const uint8_t* msg, uint64_t len, uint8_t* out64) {
    uint32_t r[8], a[8], d[16];
    b2w(r, R);
    b2w(a, A);
    hram_generic(d, r, a, msg, len);
    std::memcpy(out64, d, 64);
}

int hc_decompress(const uint8_t* in, uint8_t* out) {
    uint32_t w[8], o[8];
    b2w(w, in);
    ge_p3 p;
    const bool ok = ge_decompress(p, w);
    ge_compress_w(o, p);
    w2b(out, o);
    return ok ? 1 : 0;
}

// out: compress(a+b), compress(2a), compress(a + precomp(b)), compress(k*a)
void hc_point_ops(const uint8_t* a, const uint8_t* b, const uint8_t* k, uint8_t* sum, uint8_t* dbl, uint8_t* madd,
                  uint8_t* kmul) {
    uint32_t wa[8], wb[8], wk[8], o[8];
    b2w(wa, a);
    b2w(wb, b);
    b2w(wk, k);
    ge_p3 pa, pb;
    ge_decompress(pa, wa);
    ge_decompress(pb, wb);
    ge_compress_w(o, ge_add(pa, ge_to_cached(pb)));
    w2b(sum, o);
    ge_compress_w(o, ge_dbl(pa));
    w2b(dbl, o);
    ge_compress_w(o, ge_madd(pa, ge_precomp_cneg(ge_to_precomp(pb), false)));
    w2b(madd, o);
    ge_compress_w(o, ge_scalarmult_vartime<8>(wk, pa));
    w2b(kmul, o);
}

// The fused-carry products of k_verify's mixed addition (ge_madd<true>: fe_mul3 + fe_mul4_efgh),
// and the pair / triple / quad product groups against fe_mul on the same operands.
// out: compress(a + precomp(b)) by ge_madd<true>; returns 1 iff every grouped product equals fe_mul.
int hc_madd_fused(const uint8_t* a, const uint8_t* b, uint8_t* madd) {
    uint32_t wa[8], wb[8], o[8];
    b2w(wa, a);
    b2w(wb, b);
    ge_p3 pa, pb;
    ge_decompress(pa, wa);
    ge_decompress(pb, wb);
    const ge_precomp q = ge_precomp_cneg(ge_to_precomp(pb), false);
    ge_compress_w(o, ge_madd<true>(pa, q));
    w2b(madd, o);
    // loose operands as the addition produces them (k = 5 first operands, k <= 3 second operands)
    const fe f1 = fe_sub_loose(pa.Y, pa.X), f2 = fe_add(pa.Y, pa.X), f3 = pa.T;
    const fe g1 = q.ymx, g2 = q.ypx, g3 = fe_sub2p_loose(pa.Z, q.xy2d);
    fe h1, h2, h3, x, y, z, t;
    bool ok = true;
    auto same = [](const fe& u, const fe& v) { return fe_iszero(fe_sub(u, v)); };
    fe_mul2(h1, f1, g1, h2, f2, g2);
    ok = ok && same(h1, fe_mul(f1, g1)) && same(h2, fe_mul(f2, g2));
    fe_mul3(h1, f1, g1, h2, f2, g2, h3, f3, g3);
    ok = ok && same(h1, fe_mul(f1, g1)) && same(h2, fe_mul(f2, g2)) && same(h3, fe_mul(f3, g3));
    fe_mul4_efgh(x, y, z, t, f1, g3, f2, g2);   // e f, g h, g f, e h
    ok = ok && same(x, fe_mul(f1, g3)) && same(y, fe_mul(f2, g2)) && same(z, fe_mul(f2, g3)) && same(t, fe_mul(f1, g2));
    return ok ? 1 : 0;
}

// Build the comb table of one key exactly as k_key_prep + k_comb_entries do.
uint32_t hc_build_comb(const uint8_t* key, uint32_t* tab, int w) {
    uint32_t raw[8];
    b2w(raw, key);
    std::vector<uint32_t> bases(comb_pos(w) * 40);
    if (w == 8) return build_comb_w<8>(raw, bases.data(), tab);
    if (w == 12) return build_comb_w<12>(raw, bases.data(), tab);
    return build_comb_w<16>(raw, bases.data(), tab);
}
size_t hc_comb_words(int w) { return comb_words(w); }

// One signature through the verify lane math (single-lane inversion instead of the wave trick).
// Returns the NW_F_* flags (+ torsion coefficient bits when zseed != NULL).
uint32_t hc_verify_lane(const uint8_t* sig64, const uint8_t* pk, const uint8_t* msg, uint64_t len, uint32_t kinfo,
                        const uint32_t* atab, int wa, const uint32_t* btab, const uint8_t* zseed, uint32_t counter,
                        uint64_t bidx, uint8_t* slow_q /* 32 B compressed z(R-P) or zeros */, int* rbad) {
    uint32_t R[8], S[8], A[8];
    b2w(R, sig64);
    b2w(S, sig64 + 32);
    b2w(A, pk);
    const bool sok = sc_is_canonical(S);
    const bool aok = (kinfo & KI_OK) != 0;
    uint32_t h[8];
    if (len == 32) {
        uint32_t M[8];
        b2w(M, msg);
        hram_msg32(h, R, A, M);
    } else {
        uint32_t hw[16];
        hram_generic(hw, R, A, msg, len);
        sc_reduce512(h, hw);
    }
    const ge_p3 P = wa == 8 ? compute_P_w<8>(wa, S, h, sok, btab, atab)
                            : (wa == 12 ? compute_P_w<12>(wa, S, h, sok, btab, atab)
                                        : compute_P_w<16>(wa, S, h, sok, btab, atab));
    uint32_t flags = match_flags(P, fe_invert(P.Z), R, sok, aok, (kinfo & KI_SMALL) != 0);
    *rbad = 0;
    std::memset(slow_q, 0, 32);
    if (zseed) {
        uint32_t key[8], z4[4];
        b2w(key, zseed);
        chacha20_z(z4, key, counter, (uint32_t)bidx, (uint32_t)(bidx >> 32), 0u);
        const uint32_t tk = (kinfo >> KI_TORSION_SHIFT) & 7u;
        if (tk) flags |= torsion_coef(z4, h, tk) << NW_F_TCOEF_SHIFT;
        if (!(flags & NW_F_MATCH) && sok && aok) {
            flags |= NW_F_SLOW;
            ge_p3 Rp;
            if (!ge_decompress(Rp, R)) {
                *rbad = 1;
            } else {
                uint32_t o[8];
                ge_compress_w(o, slow_term(Rp, P, z4));
                w2b(slow_q, o);
            }
        }
    }
    return flags;
}

void hc_chacha_z(const uint8_t* key32, uint32_t counter, uint64_t bidx, uint8_t* out16) {
    uint32_t key[8], z[4];
    b2w(key, key32);
    chacha20_z(z, key, counter, (uint32_t)bidx, (uint32_t)(bidx >> 32), 0u);
    std::memcpy(out16, z, 16);
}

void hc_sign32(const uint8_t* seed, const uint8_t* msg32, const uint32_t* btab, uint8_t* pk, uint8_t* sig) {
    uint32_t s[8], m[8], p[8], g[16];
    b2w(s, seed);
    b2w(m, msg32);
    sign_one<8, 16>(s, m, btab, p, g);
    std::memcpy(pk, p, 32);
    std::memcpy(sig, g, 64);
}

}  // extern "C"
