/*
 * nw_ref.c — CPU restatement of ed25519-dalek 1.0.1 (u64 backend of curve25519-dalek 3.x) for
 * the verify hot path.  TEST / BASELINE INFRASTRUCTURE ONLY: used by tests/ (parity of the C
 * restatement against the Python oracle) and by bench.py's cpu_baseline leg.  Never linked into
 * or called by the product (narwhal_amd/).
 *
 * Follows the reference call sites:
 *   crypto::Signature::verify       (crypto/src/lib.rs:200-204)  -> nwr_verify_strict
 *   crypto::Signature::verify_batch (crypto/src/lib.rs:206-219)  -> nwr_crypto_verify_batch
 *     per vote: ed25519 Signature::from_bytes (S high bits), dalek::PublicKey::from_bytes
 *     (decompress A, every call), then dalek::verify_batch:
 *       h_i = SHA512(R||A||M) mod l; z_i 128-bit (NW-Z v1 ChaCha20 stream, replacing
 *       merlin + thread_rng); optional_multiscalar_mul over [B, R_i, A_i] with scalars
 *       [-sum z s, z_i, z_i h_i mod l] — Straus (NAF width 5) below 190 points, Pippenger
 *       (w = 6 / 7 / 8) above, exactly the size switch of curve25519-dalek 3.x — then is_identity.
 * Field: 5 x 51-bit limbs with unsigned __int128 products (FieldElement51).
 * The dalek sources are not in the container; this restates the published
 * algorithms and is pinned by tests/test_nw_ref.py against the Python oracle and golden vectors.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[5]; } fe51;

static const uint64_t MASK51 = (1ULL << 51) - 1;

/* ------------------------------------------------------------------------------- field */
static void fe_reduce(fe51* h) {
    uint64_t c;
    c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
    c = h->v[1] >> 51; h->v[1] &= MASK51; h->v[2] += c;
    c = h->v[2] >> 51; h->v[2] &= MASK51; h->v[3] += c;
    c = h->v[3] >> 51; h->v[3] &= MASK51; h->v[4] += c;
    c = h->v[4] >> 51; h->v[4] &= MASK51; h->v[0] += c * 19;
}
static fe51 fe_add(fe51 a, fe51 b) {
    fe51 r;
    for (int i = 0; i < 5; ++i) r.v[i] = a.v[i] + b.v[i];
    return r;
}
/* a - b = (a + 16p) - b, then weak reduction (dalek FieldElement51::sub) */
static fe51 fe_sub(fe51 a, fe51 b) {
    fe51 r;
    r.v[0] = (a.v[0] + 36028797018963664ULL) - b.v[0];
    for (int i = 1; i < 5; ++i) r.v[i] = (a.v[i] + 36028797018963952ULL) - b.v[i];
    fe_reduce(&r);
    return r;
}
static fe51 fe_neg(fe51 a) {
    fe51 z = {{0, 0, 0, 0, 0}};
    return fe_sub(z, a);
}
static fe51 fe_mul(fe51 a, fe51 b) {
    const uint64_t b1_19 = b.v[1] * 19, b2_19 = b.v[2] * 19, b3_19 = b.v[3] * 19, b4_19 = b.v[4] * 19;
    u128 c0 = (u128)a.v[0] * b.v[0] + (u128)a.v[4] * b1_19 + (u128)a.v[3] * b2_19 + (u128)a.v[2] * b3_19 +
              (u128)a.v[1] * b4_19;
    u128 c1 = (u128)a.v[1] * b.v[0] + (u128)a.v[0] * b.v[1] + (u128)a.v[4] * b2_19 + (u128)a.v[3] * b3_19 +
              (u128)a.v[2] * b4_19;
    u128 c2 = (u128)a.v[2] * b.v[0] + (u128)a.v[1] * b.v[1] + (u128)a.v[0] * b.v[2] + (u128)a.v[4] * b3_19 +
              (u128)a.v[3] * b4_19;
    u128 c3 = (u128)a.v[3] * b.v[0] + (u128)a.v[2] * b.v[1] + (u128)a.v[1] * b.v[2] + (u128)a.v[0] * b.v[3] +
              (u128)a.v[4] * b4_19;
    u128 c4 = (u128)a.v[4] * b.v[0] + (u128)a.v[3] * b.v[1] + (u128)a.v[2] * b.v[2] + (u128)a.v[1] * b.v[3] +
              (u128)a.v[0] * b.v[4];
    fe51 r;
    c1 += (uint64_t)(c0 >> 51); r.v[0] = (uint64_t)c0 & MASK51;
    c2 += (uint64_t)(c1 >> 51); r.v[1] = (uint64_t)c1 & MASK51;
    c3 += (uint64_t)(c2 >> 51); r.v[2] = (uint64_t)c2 & MASK51;
    c4 += (uint64_t)(c3 >> 51); r.v[3] = (uint64_t)c3 & MASK51;
    uint64_t carry = (uint64_t)(c4 >> 51); r.v[4] = (uint64_t)c4 & MASK51;
    r.v[0] += carry * 19;
    r.v[1] += r.v[0] >> 51;
    r.v[0] &= MASK51;
    return r;
}
/* dedicated squaring, 15 products (dalek FieldElement51::pow2k) */
static fe51 fe_sq(fe51 a) {
    const uint64_t a3_19 = a.v[3] * 19, a4_19 = a.v[4] * 19;
    u128 c0 = (u128)a.v[0] * a.v[0] + 2 * ((u128)a.v[1] * a4_19 + (u128)a.v[2] * a3_19);
    u128 c1 = (u128)a.v[3] * a3_19 + 2 * ((u128)a.v[0] * a.v[1] + (u128)a.v[2] * a4_19);
    u128 c2 = (u128)a.v[1] * a.v[1] + 2 * ((u128)a.v[0] * a.v[2] + (u128)a.v[4] * a3_19);
    u128 c3 = (u128)a.v[4] * a4_19 + 2 * ((u128)a.v[0] * a.v[3] + (u128)a.v[1] * a.v[2]);
    u128 c4 = (u128)a.v[2] * a.v[2] + 2 * ((u128)a.v[0] * a.v[4] + (u128)a.v[1] * a.v[3]);
    fe51 r;
    c1 += (uint64_t)(c0 >> 51); r.v[0] = (uint64_t)c0 & MASK51;
    c2 += (uint64_t)(c1 >> 51); r.v[1] = (uint64_t)c1 & MASK51;
    c3 += (uint64_t)(c2 >> 51); r.v[2] = (uint64_t)c2 & MASK51;
    c4 += (uint64_t)(c3 >> 51); r.v[3] = (uint64_t)c3 & MASK51;
    uint64_t carry = (uint64_t)(c4 >> 51); r.v[4] = (uint64_t)c4 & MASK51;
    r.v[0] += carry * 19;
    r.v[1] += r.v[0] >> 51;
    r.v[0] &= MASK51;
    return r;
}
static fe51 fe_sqn(fe51 a, int n) {
    for (int i = 0; i < n; ++i) a = fe_sq(a);
    return a;
}
static fe51 fe_from_bytes(const uint8_t b[32]) {
    uint64_t w[4];
    memcpy(w, b, 32);
    fe51 r;
    r.v[0] = w[0] & MASK51;
    r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
    r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
    r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
    r.v[4] = (w[3] >> 12) & MASK51;
    return r;
}
static void fe_to_bytes(uint8_t out[32], fe51 h) {
    fe_reduce(&h);
    /* q = floor((h + 19) / 2^255) */
    uint64_t q = (h.v[0] + 19) >> 51;
    q = (h.v[1] + q) >> 51;
    q = (h.v[2] + q) >> 51;
    q = (h.v[3] + q) >> 51;
    q = (h.v[4] + q) >> 51;
    h.v[0] += 19 * q;
    h.v[1] += h.v[0] >> 51; h.v[0] &= MASK51;
    h.v[2] += h.v[1] >> 51; h.v[1] &= MASK51;
    h.v[3] += h.v[2] >> 51; h.v[2] &= MASK51;
    h.v[4] += h.v[3] >> 51; h.v[3] &= MASK51;
    h.v[4] &= MASK51;
    uint64_t w[4];
    w[0] = h.v[0] | (h.v[1] << 51);
    w[1] = (h.v[1] >> 13) | (h.v[2] << 38);
    w[2] = (h.v[2] >> 26) | (h.v[3] << 25);
    w[3] = (h.v[3] >> 39) | (h.v[4] << 12);
    memcpy(out, w, 32);
}
static int fe_is_zero(fe51 a) {
    uint8_t b[32];
    fe_to_bytes(b, a);
    uint8_t x = 0;
    for (int i = 0; i < 32; ++i) x |= b[i];
    return x == 0;
}
static int fe_eq(fe51 a, fe51 b) { return fe_is_zero(fe_sub(a, b)); }
static int fe_is_negative(fe51 a) {
    uint8_t b[32];
    fe_to_bytes(b, a);
    return b[0] & 1;
}
static fe51 fe_pow22523(fe51 z) {
    fe51 t0 = fe_sq(z), t1 = fe_sqn(t0, 2), t2;
    t1 = fe_mul(z, t1);
    t0 = fe_mul(t0, t1);
    t0 = fe_sq(t0);
    t0 = fe_mul(t1, t0);
    t1 = fe_sqn(t0, 5);
    t0 = fe_mul(t1, t0);
    t1 = fe_sqn(t0, 10);
    t1 = fe_mul(t1, t0);
    t2 = fe_sqn(t1, 20);
    t1 = fe_mul(t2, t1);
    t1 = fe_sqn(t1, 10);
    t0 = fe_mul(t1, t0);
    t1 = fe_sqn(t0, 50);
    t1 = fe_mul(t1, t0);
    t2 = fe_sqn(t1, 100);
    t1 = fe_mul(t2, t1);
    t1 = fe_sqn(t1, 50);
    t0 = fe_mul(t1, t0);
    t0 = fe_sqn(t0, 2);
    return fe_mul(t0, z);
}
static fe51 fe_invert(fe51 z) {
    fe51 t0 = fe_sq(z), t1 = fe_sqn(t0, 2), t2, t3;
    t1 = fe_mul(z, t1);
    t0 = fe_mul(t0, t1);
    t2 = fe_sq(t0);
    t1 = fe_mul(t1, t2);
    t2 = fe_sqn(t1, 5);
    t1 = fe_mul(t2, t1);
    t2 = fe_sqn(t1, 10);
    t2 = fe_mul(t2, t1);
    t3 = fe_sqn(t2, 20);
    t2 = fe_mul(t3, t2);
    t2 = fe_sqn(t2, 10);
    t1 = fe_mul(t2, t1);
    t2 = fe_sqn(t1, 50);
    t2 = fe_mul(t2, t1);
    t3 = fe_sqn(t2, 100);
    t2 = fe_mul(t3, t2);
    t2 = fe_sqn(t2, 50);
    t1 = fe_mul(t2, t1);
    t1 = fe_sqn(t1, 5);
    return fe_mul(t1, t0);
}

static fe51 FE_ONE = {{1, 0, 0, 0, 0}};
static fe51 FE_ZERO = {{0, 0, 0, 0, 0}};
static fe51 FE_D, FE_D2, FE_SQRTM1;
static uint8_t L_BYTES[32];

/* ------------------------------------------------------------------------------- points */
typedef struct { fe51 X, Y, Z, T; } ge;          /* extended */
typedef struct { fe51 YpX, YmX, Z, T2d; } ge_pn;  /* projective Niels */
typedef struct { fe51 X, Y, Z, T; } ge_c;         /* completed ((X:Z),(Y:T)) */

static ge ge_identity(void) {
    ge r = {FE_ZERO, FE_ONE, FE_ONE, FE_ZERO};
    return r;
}
static ge_pn ge_to_pn(const ge* p) {
    ge_pn r;
    r.YpX = fe_add(p->Y, p->X);
    r.YmX = fe_sub(p->Y, p->X);
    r.Z = p->Z;
    r.T2d = fe_mul(p->T, FE_D2);
    return r;
}
static ge ge_from_c(const ge_c* c) {
    ge r;
    r.X = fe_mul(c->X, c->T);
    r.Y = fe_mul(c->Y, c->Z);
    r.Z = fe_mul(c->Z, c->T);
    r.T = fe_mul(c->X, c->Y);
    return r;
}
/* projective-only conversion (drops T) for doubling chains, as dalek's ProjectivePoint */
static ge ge_from_c_proj(const ge_c* c) {
    ge r;
    r.X = fe_mul(c->X, c->T);
    r.Y = fe_mul(c->Y, c->Z);
    r.Z = fe_mul(c->Z, c->T);
    r.T = FE_ZERO;
    return r;
}
static ge_c ge_add_pn(const ge* p, const ge_pn* q) {
    fe51 ypx = fe_add(p->Y, p->X), ymx = fe_sub(p->Y, p->X);
    fe51 pp = fe_mul(ypx, q->YpX), mm = fe_mul(ymx, q->YmX);
    fe51 tt2d = fe_mul(p->T, q->T2d);
    fe51 zz = fe_mul(p->Z, q->Z);
    fe51 zz2 = fe_add(zz, zz);
    ge_c r;
    r.X = fe_sub(pp, mm);
    r.Y = fe_add(pp, mm);
    r.Z = fe_add(zz2, tt2d);
    r.T = fe_sub(zz2, tt2d);
    return r;
}
static ge_c ge_sub_pn(const ge* p, const ge_pn* q) {
    fe51 ypx = fe_add(p->Y, p->X), ymx = fe_sub(p->Y, p->X);
    fe51 pm = fe_mul(ypx, q->YmX), mp = fe_mul(ymx, q->YpX);
    fe51 tt2d = fe_mul(p->T, q->T2d);
    fe51 zz = fe_mul(p->Z, q->Z);
    fe51 zz2 = fe_add(zz, zz);
    ge_c r;
    r.X = fe_sub(pm, mp);
    r.Y = fe_add(pm, mp);
    r.Z = fe_sub(zz2, tt2d);
    r.T = fe_add(zz2, tt2d);
    return r;
}
/* doubling from projective (X:Y:Z) -> completed (dalek ProjectivePoint::double) */
static ge_c ge_double_c(const ge* p) {
    fe51 xx = fe_sq(p->X), yy = fe_sq(p->Y), zz2 = fe_sq(p->Z);
    zz2 = fe_add(zz2, zz2);
    fe51 xpy = fe_add(p->X, p->Y), xpy2 = fe_sq(xpy);
    fe51 yypxx = fe_add(yy, xx), yymxx = fe_sub(yy, xx);
    ge_c r;
    r.X = fe_sub(xpy2, yypxx);
    r.Y = yypxx;
    r.Z = yymxx;
    r.T = fe_sub(zz2, yymxx);
    return r;
}
static ge ge_add(const ge* p, const ge* q) {
    ge_pn qn = ge_to_pn(q);
    ge_c c = ge_add_pn(p, &qn);
    return ge_from_c(&c);
}
static ge ge_dbl(const ge* p) {
    ge_c c = ge_double_c(p);
    return ge_from_c(&c);
}
static int ge_is_identity(const ge* p) { return fe_is_zero(p->X) && fe_eq(p->Y, p->Z); }
static int ge_eq(const ge* p, const ge* q) {
    return fe_eq(fe_mul(p->X, q->Z), fe_mul(q->X, p->Z)) && fe_eq(fe_mul(p->Y, q->Z), fe_mul(q->Y, p->Z));
}
static int ge_is_small_order(const ge* p) {
    ge t = ge_dbl(p);
    t = ge_dbl(&t);
    t = ge_dbl(&t);
    return ge_is_identity(&t);
}

/* CompressedEdwardsY::decompress (dalek): y mod p without rejecting y >= p; sign of x from bit 255 */
static int ge_decompress(ge* out, const uint8_t b[32]) {
    fe51 y = fe_from_bytes(b);
    fe51 yy = fe_sq(y);
    fe51 u = fe_sub(yy, FE_ONE);
    fe51 v = fe_add(fe_mul(yy, FE_D), FE_ONE);
    fe51 v3 = fe_mul(fe_sq(v), v);
    fe51 v7 = fe_mul(fe_sq(v3), v);
    fe51 r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
    fe51 check = fe_mul(v, fe_sq(r));
    fe51 nu = fe_neg(u);
    int correct = fe_eq(check, u), flipped = fe_eq(check, nu), flipped_i = fe_eq(check, fe_mul(nu, FE_SQRTM1));
    if (flipped || flipped_i) r = fe_mul(r, FE_SQRTM1);
    if (fe_is_negative(r)) r = fe_neg(r);
    if (!(correct || flipped)) return 0;
    if (b[31] >> 7) r = fe_neg(r);
    out->X = r;
    out->Y = y;
    out->Z = FE_ONE;
    out->T = fe_mul(r, y);
    return 1;
}

/* ------------------------------------------------------------------------------- SHA-512 */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void sha512_block(uint64_t st[8], const uint8_t* p) {
    uint64_t w[80];
    for (int i = 0; i < 16; ++i) {
        uint64_t x = 0;
        for (int j = 0; j < 8; ++j) x = (x << 8) | p[8 * i + j];
        w[i] = x;
    }
    for (int i = 16; i < 80; ++i) {
        uint64_t s0 = ROR64(w[i - 15], 1) ^ ROR64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = ROR64(w[i - 2], 19) ^ ROR64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 80; ++i) {
        uint64_t t1 = h + (ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
        uint64_t t2 = (ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* SHA-512 over the concatenation of up to 3 buffers */
static void sha512_3(uint8_t out[64], const uint8_t* a, size_t al, const uint8_t* b, size_t bl, const uint8_t* c,
                     size_t cl) {
    uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                      0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    uint8_t blk[128];
    size_t fill = 0;
    const uint8_t* parts[3] = {a, b, c};
    size_t lens[3] = {al, bl, cl};
    uint64_t total = al + bl + cl;
    for (int k = 0; k < 3; ++k) {
        const uint8_t* p = parts[k];
        size_t n = lens[k];
        while (n) {
            size_t take = 128 - fill < n ? 128 - fill : n;
            memcpy(blk + fill, p, take);
            fill += take;
            p += take;
            n -= take;
            if (fill == 128) {
                sha512_block(st, blk);
                fill = 0;
            }
        }
    }
    blk[fill++] = 0x80;
    if (fill > 112) {
        memset(blk + fill, 0, 128 - fill);
        sha512_block(st, blk);
        fill = 0;
    }
    memset(blk + fill, 0, 128 - fill);
    uint64_t bits = total * 8;
    for (int j = 0; j < 8; ++j) blk[127 - j] = (uint8_t)(bits >> (8 * j));
    sha512_block(st, blk);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(st[i] >> (56 - 8 * j));
}

/* ------------------------------------------------------------------------------- scalars */
static const uint32_t SC_L32[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0, 0, 0, 0x10000000};
static const uint32_t SC_MU32[9] = {0x0a2c131b, 0xed9ce5a3, 0x086329a7, 0x2106215d, 0xffffffeb,
                                    0xffffffff, 0xffffffff, 0xffffffff, 0x0000000f};

static void mulw(uint32_t* r, const uint32_t* a, int na, const uint32_t* b, int nb) {
    memset(r, 0, sizeof(uint32_t) * (na + nb));
    for (int i = 0; i < na; ++i) {
        uint64_t carry = 0;
        for (int j = 0; j < nb; ++j) {
            uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + carry;
            r[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        r[i + nb] = (uint32_t)carry;
    }
}
static int geq8(const uint32_t* a, const uint32_t* b) {
    for (int i = 7; i >= 0; --i) {
        if (a[i] > b[i]) return 1;
        if (a[i] < b[i]) return 0;
    }
    return 1;
}
static void sub8(uint32_t* r, const uint32_t* a, const uint32_t* b) {
    uint64_t borrow = 0;
    for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)a[i] - b[i] - borrow;
        r[i] = (uint32_t)t;
        borrow = (t >> 63) & 1;
    }
}
/* x (16 words) mod l -> 32 bytes */
static void sc_reduce512(uint8_t out[32], const uint32_t x[16]) {
    uint32_t q2[18], q3[9], r2[18], r[9];
    mulw(q2, x + 7, 9, SC_MU32, 9);
    memcpy(q3, q2 + 9, 36);
    mulw(r2, q3, 9, SC_L32, 8);
    uint64_t borrow = 0;
    for (int i = 0; i < 9; ++i) {
        uint64_t t = (uint64_t)x[i] - r2[i] - borrow;
        r[i] = (uint32_t)t;
        borrow = (t >> 63) & 1;
    }
    for (int k = 0; k < 2; ++k)
        if (geq8(r, SC_L32)) sub8(r, r, SC_L32);
    memcpy(out, r, 32);
}
static void sc_from_hash(uint8_t out[32], const uint8_t h[64]) {
    uint32_t x[16];
    memcpy(x, h, 64);
    sc_reduce512(out, x);
}
static void sc_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
    uint32_t x[8], y[8], p[16];
    memcpy(x, a, 32);
    memcpy(y, b, 32);
    mulw(p, x, 8, y, 8);
    sc_reduce512(out, p);
}
static void sc_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
    uint32_t x[16] = {0}, y[8];
    memcpy(x, a, 32);
    memcpy(y, b, 32);
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
        uint64_t t = (uint64_t)x[i] + y[i] + c;
        x[i] = (uint32_t)t;
        c = t >> 32;
    }
    x[8] = (uint32_t)c;
    sc_reduce512(out, x);
}
static void sc_neg(uint8_t out[32], const uint8_t a[32]) {
    uint32_t x[8], r[8];
    memcpy(x, a, 32);
    int zero = 1;
    for (int i = 0; i < 8; ++i) zero &= x[i] == 0;
    if (zero) {
        memset(out, 0, 32);
        return;
    }
    sub8(r, SC_L32, x);
    memcpy(out, r, 32);
}
/* S < l (ed25519 high-3-bit check + dalek check_scalar) */
static int sc_canonical(const uint8_t s[32]) {
    if (s[31] & 0xE0) return 0;
    uint32_t x[8];
    memcpy(x, s, 32);
    return !geq8(x, SC_L32);
}

/* width-w NAF of a 256-bit little-endian scalar (dalek Scalar::non_adjacent_form) */
static void naf(int8_t out[256], const uint8_t s[32], int w) {
    uint64_t x[5] = {0, 0, 0, 0, 0};
    memcpy(x, s, 32);
    memset(out, 0, 256);
    const uint64_t width = 1ULL << w, window_mask = width - 1;
    size_t pos = 0;
    uint64_t carry = 0;
    while (pos < 256) {
        size_t idx = pos / 64, bit = pos % 64;
        uint64_t bit_buf = bit < 64 - w ? x[idx] >> bit : (x[idx] >> bit) | (x[1 + idx] << (64 - bit));
        uint64_t window = carry + (bit_buf & window_mask);
        if ((window & 1) == 0) {
            pos += 1;
            continue;
        }
        if (window < width / 2) {
            carry = 0;
            out[pos] = (int8_t)window;
        } else {
            carry = 1;
            out[pos] = (int8_t)((int64_t)window - (int64_t)width);
        }
        pos += w;
    }
}

/* signed radix-2^w digits (dalek Scalar::to_radix_2w), digits in [-2^(w-1), 2^(w-1)] */
static int radix2w(int8_t* out, const uint8_t s[32], int w) {
    uint64_t x[4];
    memcpy(x, s, 32);
    const int digits_count = (256 + w - 1) / w;
    const uint64_t radix = 1ULL << w, window_mask = radix - 1;
    int64_t carry = 0;
    for (int i = 0; i < digits_count; ++i) {
        int bit_offset = i * w;
        int u64_idx = bit_offset / 64, bit_idx = bit_offset % 64;
        uint64_t bit_buf;
        if (bit_idx < 64 - w || u64_idx == 3)
            bit_buf = x[u64_idx] >> bit_idx;
        else
            bit_buf = (x[u64_idx] >> bit_idx) | (x[1 + u64_idx] << (64 - bit_idx));
        int64_t coef = carry + (int64_t)(bit_buf & window_mask);
        carry = (coef + (int64_t)(radix / 2)) >> w;
        out[i] = (int8_t)(coef - (carry << w));
    }
    out[digits_count - 1] += (int8_t)(carry << w);
    return digits_count;
}

/* ------------------------------------------------------------------------------- MSM */
typedef struct { ge_pn t[8]; } naf_table5;   /* P, 3P, ..., 15P */

static void make_naf_table5(naf_table5* tb, const ge* p) {
    ge p2 = ge_dbl(p);
    ge cur = *p;
    for (int i = 0; i < 8; ++i) {
        tb->t[i] = ge_to_pn(&cur);
        cur = ge_add(&cur, &p2);
    }
}

/* Straus (dalek VartimeMultiscalarMul for n < 190): sum s_i P_i.  As in dalek, the accumulator
 * stays projective across doublings and is extended only when a table entry is added. */
static ge msm_straus(const uint8_t (*sc)[32], const ge* pts, size_t n, int8_t* nafs, naf_table5* tabs) {
    for (size_t i = 0; i < n; ++i) {
        naf(nafs + 256 * i, sc[i], 5);
        make_naf_table5(&tabs[i], &pts[i]);
    }
    ge r = ge_identity();
    for (int b = 255; b >= 0; --b) {
        ge_c t = ge_double_c(&r);
        for (size_t i = 0; i < n; ++i) {
            int8_t d = nafs[256 * i + b];
            if (d > 0) {
                ge e = ge_from_c(&t);
                t = ge_add_pn(&e, &tabs[i].t[d / 2]);
            } else if (d < 0) {
                ge e = ge_from_c(&t);
                t = ge_sub_pn(&e, &tabs[i].t[(-d) / 2]);
            }
        }
        r = ge_from_c_proj(&t);
    }
    return r;   /* projective: callers only use X, Y, Z (ge_eq / ge_is_identity) */
}

/* Pippenger (dalek Pippenger::optional_multiscalar_mul): w = 6 (<500), 7 (<800), 8 otherwise */
static ge msm_pippenger(const uint8_t (*sc)[32], const ge* pts, size_t n) {
    const int w = n < 500 ? 6 : (n < 800 ? 7 : 8);
    const int max_digit = 1 << (w - 1);
    const int digits_count = (256 + w - 1) / w;
    const int nb = max_digit;
    int8_t* digits = (int8_t*)malloc((size_t)n * digits_count);
    ge_pn* pn = (ge_pn*)malloc(sizeof(ge_pn) * n);
    ge* buckets = (ge*)malloc(sizeof(ge) * nb);
    for (size_t i = 0; i < n; ++i) {
        radix2w(digits + (size_t)i * digits_count, sc[i], w);
        pn[i] = ge_to_pn(&pts[i]);
    }
    ge total = ge_identity();
    for (int dig = digits_count - 1; dig >= 0; --dig) {
        for (int b = 0; b < nb; ++b) buckets[b] = ge_identity();
        for (size_t i = 0; i < n; ++i) {
            int8_t d = digits[(size_t)i * digits_count + dig];
            if (d > 0) {
                ge_c t = ge_add_pn(&buckets[d - 1], &pn[i]);
                buckets[d - 1] = ge_from_c(&t);
            } else if (d < 0) {
                ge_c t = ge_sub_pn(&buckets[-d - 1], &pn[i]);
                buckets[-d - 1] = ge_from_c(&t);
            }
        }
        ge running = buckets[nb - 1], sum = buckets[nb - 1];
        for (int b = nb - 2; b >= 0; --b) {
            running = ge_add(&running, &buckets[b]);
            sum = ge_add(&sum, &running);
        }
        for (int k = 0; k < w; ++k) total = ge_dbl(&total);
        total = ge_add(&total, &sum);
    }
    free(digits);
    free(pn);
    free(buckets);
    return total;
}

/* ------------------------------------------------------------------------------- ChaCha20 z */
static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d) a += b; d = rotl32(d ^ a, 16); c += d; b = rotl32(b ^ c, 12); \
                       a += b; d = rotl32(d ^ a, 8);  c += d; b = rotl32(b ^ c, 7)
static void nwz(uint8_t z[32], const uint8_t key[32], uint32_t counter, uint64_t bidx) {
    uint32_t k[8], x[16], s[16];
    memcpy(k, key, 32);
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; ++i) s[4 + i] = k[i];
    s[12] = counter; s[13] = (uint32_t)bidx; s[14] = (uint32_t)(bidx >> 32); s[15] = 0;
    memcpy(x, s, 64);
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]); QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]); QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    uint32_t out[4];
    for (int i = 0; i < 4; ++i) out[i] = x[i] + s[i];
    memset(z, 0, 32);
    memcpy(z, out, 16);
}

/* ------------------------------------------------------------------------------- API */
static ge GE_B;
typedef struct { fe51 YpX, YmX, XY2d; } ge_an;   /* affine Niels (dalek AffineNielsPoint) */
static ge_an B_ODD[64];                            /* B, 3B, ..., 127B */
static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void init_consts(void) {
    static const uint8_t d_bytes[32] = {0xa3, 0x78, 0x59, 0x13, 0xca, 0x4d, 0xeb, 0x75, 0xab, 0xd8, 0x41,
                                        0x41, 0x4d, 0x0a, 0x70, 0x00, 0x98, 0xe8, 0x79, 0x77, 0x79, 0x40,
                                        0xc7, 0x8c, 0x73, 0xfe, 0x6f, 0x2b, 0xee, 0x6c, 0x03, 0x52};
    static const uint8_t sqrtm1_bytes[32] = {0xb0, 0xa0, 0x0e, 0x4a, 0x27, 0x1b, 0xee, 0xc4, 0x78, 0xe4, 0x2f,
                                             0xad, 0x06, 0x18, 0x43, 0x2f, 0xa7, 0xd7, 0xfb, 0x3d, 0x99, 0x00,
                                             0x4d, 0x2b, 0x0b, 0xdf, 0xc1, 0x4f, 0x80, 0x24, 0x83, 0x2b};
    static const uint8_t b_bytes[32] = {0x58, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                        0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66,
                                        0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66, 0x66};
    FE_D = fe_from_bytes(d_bytes);
    FE_D2 = fe_add(FE_D, FE_D);
    fe_reduce(&FE_D2);
    FE_SQRTM1 = fe_from_bytes(sqrtm1_bytes);
    ge_decompress(&GE_B, b_bytes);
    {
        ge b2 = ge_dbl(&GE_B), cur = GE_B;
        for (int i = 0; i < 64; ++i) {
            fe51 zi = fe_invert(cur.Z);
            fe51 x = fe_mul(cur.X, zi), y = fe_mul(cur.Y, zi);
            B_ODD[i].YpX = fe_add(y, x);
            B_ODD[i].YmX = fe_sub(y, x);
            B_ODD[i].XY2d = fe_mul(fe_mul(x, y), FE_D2);
            cur = ge_add(&cur, &b2);
        }
    }
    memcpy(L_BYTES, SC_L32, 32);
}

void nwr_init(void) { pthread_once(&init_once, init_consts); }

void nwr_sha512(const uint8_t* m, size_t len, uint8_t out[64]) { sha512_3(out, m, len, 0, 0, 0, 0); }

int nwr_decompress(const uint8_t in[32], uint8_t out_canonical[32]) {
    nwr_init();
    ge p;
    if (!ge_decompress(&p, in)) return 0;
    fe51 zi = fe_invert(p.Z);
    uint8_t xb[32];
    fe_to_bytes(xb, fe_mul(p.X, zi));
    fe_to_bytes(out_canonical, fe_mul(p.Y, zi));
    out_canonical[31] |= (uint8_t)((xb[0] & 1) << 7);
    return 1;
}

/* dalek PublicKey::verify_strict.  R = [k](-A) + [s]B by dalek's serial
 * vartime_double_base::mul (curve25519-dalek 3.x, the precomputed-tables default): width-5 NAF of k
 * over a per-call projective Niels table of -A, width-8 NAF of s over the precomputed affine Niels
 * odd multiples of B (AFFINE_ODD_MULTIPLES_OF_BASEPOINT), the loop starting at the highest nonzero
 * digit of either.  The result point is algorithm-independent; the shape matters for the latency
 * comparator (bench.py cpu_baseline.latency). */
static ge_c ge_add_an(const ge* p, const ge_an* q) {
    fe51 ypx = fe_add(p->Y, p->X), ymx = fe_sub(p->Y, p->X);
    fe51 pp = fe_mul(ypx, q->YpX), mm = fe_mul(ymx, q->YmX);
    fe51 txy2d = fe_mul(p->T, q->XY2d);
    fe51 z2 = fe_add(p->Z, p->Z);
    ge_c r;
    r.X = fe_sub(pp, mm);
    r.Y = fe_add(pp, mm);
    r.Z = fe_add(z2, txy2d);
    r.T = fe_sub(z2, txy2d);
    return r;
}
static ge_c ge_sub_an(const ge* p, const ge_an* q) {
    fe51 ypx = fe_add(p->Y, p->X), ymx = fe_sub(p->Y, p->X);
    fe51 pm = fe_mul(ypx, q->YmX), mp = fe_mul(ymx, q->YpX);
    fe51 txy2d = fe_mul(p->T, q->XY2d);
    fe51 z2 = fe_add(p->Z, p->Z);
    ge_c r;
    r.X = fe_sub(pm, mp);
    r.Y = fe_add(pm, mp);
    r.Z = fe_sub(z2, txy2d);
    r.T = fe_add(z2, txy2d);
    return r;
}

static ge double_base_vartime(const uint8_t a[32], const ge* A, const uint8_t b[32]) {
    int8_t an[256], bn[256];
    naf(an, a, 5);
    naf(bn, b, 8);
    int i = 255;
    while (i > 0 && an[i] == 0 && bn[i] == 0) --i;
    naf_table5 ta;
    make_naf_table5(&ta, A);
    ge r = ge_identity();
    for (;; --i) {
        ge_c t = ge_double_c(&r);
        if (an[i] > 0) {
            ge e = ge_from_c(&t);
            t = ge_add_pn(&e, &ta.t[an[i] / 2]);
        } else if (an[i] < 0) {
            ge e = ge_from_c(&t);
            t = ge_sub_pn(&e, &ta.t[(-an[i]) / 2]);
        }
        if (bn[i] > 0) {
            ge e = ge_from_c(&t);
            t = ge_add_an(&e, &B_ODD[bn[i] / 2]);
        } else if (bn[i] < 0) {
            ge e = ge_from_c(&t);
            t = ge_sub_an(&e, &B_ODD[(-bn[i]) / 2]);
        }
        r = ge_from_c_proj(&t);
        if (i == 0) break;
    }
    return r;   /* projective: ge_eq uses X, Y, Z only */
}

int nwr_verify_strict(const uint8_t* msg, size_t len, const uint8_t pk[32], const uint8_t sig[64]) {
    nwr_init();
    if (!sc_canonical(sig + 32)) return 0;
    ge A, R;
    if (!ge_decompress(&A, pk)) return 0;
    if (!ge_decompress(&R, sig)) return 0;
    if (ge_is_small_order(&R) || ge_is_small_order(&A)) return 0;
    uint8_t h[64], k[32];
    sha512_3(h, sig, 32, pk, 32, msg, len);
    sc_from_hash(k, h);
    ge mA = A;
    mA.X = fe_neg(A.X);
    mA.T = fe_neg(A.T);
    ge Rp = double_base_vartime(k, &mA, sig + 32);
    return ge_eq(&Rp, &R);
}

/* dalek::verify_batch core: signature i over msgs[i] (lens[i] bytes).  Key decompression per
 * call (crypto/src/lib.rs:216 for certificates; dalek PublicKey values for the worker). */
static int verify_batch_core(const uint8_t* const* msgs, const size_t* lens, const uint8_t (*pk)[32],
                             const uint8_t (*sig)[64], size_t n, const uint8_t zseed[32], uint64_t bidx);

/* crypto::Signature::verify_batch over one certificate: votes (pk_i, sig_i) all over msg.
 * Per-vote key decompression as crypto/src/lib.rs:216.  Returns 1 (Ok) / 0 (Err). */
int nwr_crypto_verify_batch(const uint8_t* msg, size_t len, const uint8_t (*pk)[32], const uint8_t (*sig)[64],
                            size_t n, const uint8_t zseed[32], uint64_t bidx) {
    nwr_init();
    const uint8_t** msgs = (const uint8_t**)malloc(sizeof(uint8_t*) * (n ? n : 1));
    size_t* lens = (size_t*)malloc(sizeof(size_t) * (n ? n : 1));
    for (size_t i = 0; i < n; ++i) {
        msgs[i] = msg;
        lens[i] = len;
    }
    const int ok = verify_batch_core(msgs, lens, pk, sig, n, zseed, bidx);
    free(msgs);
    free(lens);
    return ok;
}

/* ed25519_dalek::verify_batch with per-signature messages (worker/src/processor.rs:78). */
int nwr_verify_batch_msgs(const uint8_t* const* msgs, const size_t* lens, const uint8_t (*pk)[32],
                          const uint8_t (*sig)[64], size_t n, const uint8_t zseed[32], uint64_t bidx) {
    nwr_init();
    return verify_batch_core(msgs, lens, pk, sig, n, zseed, bidx);
}

static int verify_batch_core(const uint8_t* const* msgs, const size_t* lens, const uint8_t (*pk)[32],
                             const uint8_t (*sig)[64], size_t n, const uint8_t zseed[32], uint64_t bidx) {
    for (size_t i = 0; i < n; ++i)
        if (sig[i][63] & 0xE0) return 0;
    const size_t npts = 2 * n + 1;
    ge* pts = (ge*)malloc(sizeof(ge) * npts);
    uint8_t (*sc)[32] = (uint8_t (*)[32])malloc(32 * npts);
    int ok = 1;
    for (size_t i = 0; i < n && ok; ++i)
        if (!ge_decompress(&pts[1 + n + i], pk[i])) ok = 0;      /* dalek::PublicKey::from_bytes */
    for (size_t i = 0; i < n && ok; ++i)
        if (!sc_canonical(sig[i] + 32)) ok = 0;                   /* InternalSignature::try_from */
    uint8_t bsum[32] = {0};
    for (size_t i = 0; i < n && ok; ++i) {
        uint8_t h[64], hr[32], z[32], zs[32];
        sha512_3(h, sig[i], 32, pk[i], 32, msgs[i], lens[i]);
        sc_from_hash(hr, h);
        nwz(z, zseed, (uint32_t)i, bidx);
        sc_mul(zs, z, sig[i] + 32);
        sc_add(bsum, bsum, zs);
        memcpy(sc[1 + i], z, 32);
        sc_mul(sc[1 + n + i], z, hr);
        if (!ge_decompress(&pts[1 + i], sig[i])) ok = 0;          /* R decompression */
    }
    if (ok) {
        sc_neg(sc[0], bsum);
        pts[0] = GE_B;
        ge id;
        if (npts < 190) {
            int8_t* nafs = (int8_t*)malloc(256 * npts);
            naf_table5* tabs = (naf_table5*)malloc(sizeof(naf_table5) * npts);
            id = msm_straus((const uint8_t(*)[32])sc, pts, npts, nafs, tabs);
            free(nafs);
            free(tabs);
        } else {
            id = msm_pippenger((const uint8_t(*)[32])sc, pts, npts);
        }
        ok = ge_is_identity(&id);
    }
    free(pts);
    free(sc);
    return ok;
}

/* ---- multi-threaded certificate driver (the CPU baseline) ---- */
typedef struct {
    const uint8_t* msgs;        /* [ncert][32] */
    const uint32_t* first;      /* [ncert] */
    const uint32_t* nvotes;     /* [ncert] */
    const uint8_t* pks;         /* committee [K][32] */
    const uint32_t* signer;     /* [nsig] */
    const uint8_t* sigs;        /* [nsig][64] */
    const uint32_t* sel;        /* selected certificates */
    size_t nsel;
    const uint8_t* zseed;
    uint64_t cert_base;
    uint8_t* out;
    size_t next;
    pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    uint8_t (*pk)[32] = NULL;
    size_t cap = 0;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        size_t k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->nsel) break;
        uint32_t c = j->sel[k], f = j->first[c], n = j->nvotes[c];
        if (n > cap) {
            free(pk);
            cap = n;
            pk = (uint8_t (*)[32])malloc(32 * (size_t)cap);
        }
        for (uint32_t v = 0; v < n; ++v) memcpy(pk[v], j->pks + 32 * (size_t)j->signer[f + v], 32);
        j->out[k] = (uint8_t)nwr_crypto_verify_batch(j->msgs + 32 * (size_t)c, 32, (const uint8_t(*)[32])pk,
                                                     (const uint8_t(*)[64])(j->sigs + 64 * (size_t)f), n, j->zseed,
                                                     j->cert_base + c);
    }
    free(pk);
    return NULL;
}

int nwr_verify_certs(const uint8_t* msgs, const uint32_t* first, const uint32_t* nvotes, const uint8_t* pks,
                     const uint32_t* signer, const uint8_t* sigs, const uint32_t* sel, size_t nsel,
                     const uint8_t zseed[32], uint64_t cert_base, int threads, uint8_t* out) {
    nwr_init();
    job_t j = {msgs, first, nvotes, pks, signer, sigs, sel, nsel, zseed, cert_base, out, 0};
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
    return 0;
}
