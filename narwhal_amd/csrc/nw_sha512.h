// SHA-512 (FIPS 180-4) for gfx950: replaces sha2 0.9 ``Sha512`` reached through
// ``ed25519_dalek::Sha512`` (primary/src/messages.rs:72,147,228; worker/src/processor.rs:65;
// worker/src/batch_maker.rs:125) and the hram hash inside dalek's verify paths.
//
// 64-bit words live in VGPR pairs; rotates are funnel shifts (v_alignbit_b32 pairs).  The 80
// rounds run as 5 rolled iterations of a 16-round unrolled body so the message schedule stays in
// registers (no runtime-indexed arrays) and the round constants are wave-uniform scalar loads.
#pragma once
#include <cstdint>
#include "nw_field.h"

namespace nw {

static constexpr uint64_t SHA512_K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

static constexpr uint64_t SHA512_IV[8] = {
    0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
    0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

// 64-bit rotate as two funnel shifts (v_alignbit_b32) on the device: the generic rotate lowers to
// v_lshrrev_b64 + v_lshlrev_b64 + 2 x v_or_b32, twice the instructions.  n is a compile-time
// constant at every call site, so the half swap for n >= 32 folds away.
NW_HD uint64_t rotr64(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (n >= 32) {
        const uint32_t t = lo;
        lo = hi;
        hi = t;
        n -= 32;
    }
    const uint32_t rlo = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)n);
    const uint32_t rhi = __builtin_amdgcn_alignbit(lo, hi, (uint32_t)n);
    return ((uint64_t)rhi << 32) | rlo;
#else
    return __builtin_rotateright64(x, n);
#endif
}

NW_HD uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Three-input bit functions as one gfx950 v_bitop3_b32 per 32-bit half (truth table over
// S0 = 0xF0, S1 = 0xCC, S2 = 0xAA): the compiler emits two or three 2-input ops per half for them.
template <int TT>
NW_HD uint64_t bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t lo, hi;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4"
        : "=v"(lo) : "v"((uint32_t)a), "v"((uint32_t)b), "v"((uint32_t)c), "i"(TT));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4"
        : "=v"(hi) : "v"((uint32_t)(a >> 32)), "v"((uint32_t)(b >> 32)), "v"((uint32_t)(c >> 32)), "i"(TT));
    uint64_t r = ((uint64_t)hi << 32) | lo;
    asm("" : "+v"(r));   // opaque: keeps LLVM from splitting later 64-bit adds over the halves
    return r;
#else
    uint64_t r = 0;
    for (int bit = 0; bit < 64; ++bit) {
        const int idx = (int)(((a >> bit) & 1) << 2 | ((b >> bit) & 1) << 1 | ((c >> bit) & 1));
        r |= (uint64_t)((TT >> idx) & 1) << bit;
    }
    return r;
#endif
}

NW_HD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) { return bitop3_64<0x96>(a, b, c); }

// Maj(a, b, c) = (a & b) | (a & c) | (b & c)
NW_HD uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) { return bitop3_64<0xE8>(a, b, c); }

// Ch(e, f, g) = (e & f) ^ (~e & g) as one bitop3 per half (LLVM otherwise splits it into an AND and
// a BFI whose disjoint halves it then adds separately)
NW_HD uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) { return bitop3_64<0xCA>(e, f, g); }

// big-endian 64-bit word from two little-endian-loaded u32 (bytes b0..b3 in lo, b4..b7 in hi)
NW_HD uint64_t be64_from_le32(uint32_t lo, uint32_t hi) {
    return ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
}

#define NW_SHA_ROUND(a, b, c, d, e, f, g, h, k, w)                                        \
    do {                                                                                    \
        const uint64_t t1 = (h) + xor3_64(rotr64((e), 14), rotr64((e), 18), rotr64((e), 41)) + \
                            ch64((e), (f), (g)) + (k) + (w);                       \
        const uint64_t t2 = xor3_64(rotr64((a), 28), rotr64((a), 34), rotr64((a), 39)) +   \
                            maj64((a), (b), (c));                                           \
        (d) += t1;                                                                          \
        (h) = t1 + t2;                                                                      \
    } while (0)

// One compression of a 128-byte block given as 16 big-endian words.
NW_HD void sha512_compress(uint64_t st[8], const uint64_t win[16]) {
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = win[i];
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma nounroll
    for (int r = 0; r < 80; r += 16) {
        if (r > 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
                const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), w15 >> 7);
                const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), w2 >> 6);
                w[i] += s0 + w[(i + 9) & 15] + s1;
            }
        }
        NW_SHA_ROUND(a, b, c, d, e, f, g, h, SHA512_K[r + 0], w[0]);
        NW_SHA_ROUND(h, a, b, c, d, e, f, g, SHA512_K[r + 1], w[1]);
        NW_SHA_ROUND(g, h, a, b, c, d, e, f, SHA512_K[r + 2], w[2]);
        NW_SHA_ROUND(f, g, h, a, b, c, d, e, SHA512_K[r + 3], w[3]);
        NW_SHA_ROUND(e, f, g, h, a, b, c, d, SHA512_K[r + 4], w[4]);
        NW_SHA_ROUND(d, e, f, g, h, a, b, c, SHA512_K[r + 5], w[5]);
        NW_SHA_ROUND(c, d, e, f, g, h, a, b, SHA512_K[r + 6], w[6]);
        NW_SHA_ROUND(b, c, d, e, f, g, h, a, SHA512_K[r + 7], w[7]);
        NW_SHA_ROUND(a, b, c, d, e, f, g, h, SHA512_K[r + 8], w[8]);
        NW_SHA_ROUND(h, a, b, c, d, e, f, g, SHA512_K[r + 9], w[9]);
        NW_SHA_ROUND(g, h, a, b, c, d, e, f, SHA512_K[r + 10], w[10]);
        NW_SHA_ROUND(f, g, h, a, b, c, d, e, SHA512_K[r + 11], w[11]);
        NW_SHA_ROUND(e, f, g, h, a, b, c, d, SHA512_K[r + 12], w[12]);
        NW_SHA_ROUND(d, e, f, g, h, a, b, c, SHA512_K[r + 13], w[13]);
        NW_SHA_ROUND(c, d, e, f, g, h, a, b, SHA512_K[r + 14], w[14]);
        NW_SHA_ROUND(b, c, d, e, f, g, h, a, SHA512_K[r + 15], w[15]);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

NW_HD void sha512_init(uint64_t st[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = SHA512_IV[i];
}

// Digest as 16 little-endian u32 words of the 64-byte output string (the layout
// Scalar::from_hash reads as a 512-bit LE integer).
NW_HD void sha512_digest_le32(uint32_t out[16], const uint64_t st[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        out[2 * i] = bswap32((uint32_t)(st[i] >> 32));
        out[2 * i + 1] = bswap32((uint32_t)st[i]);
    }
}

// SHA-512 of a message of 12 little-endian u32 words (48 bytes) .. up to 27 words (108 bytes):
// the single-block case. ``nwords`` must be a compile-time constant at every call site.
template <int NWORDS>
NW_HD void sha512_oneblock_le32(uint32_t out[16], const uint32_t msg[NWORDS]) {
    static_assert(NWORDS * 4 <= 111, "single-block SHA-512 needs len <= 111 bytes");
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int lo = 2 * i, hi = 2 * i + 1;
        const uint32_t wl = lo < NWORDS ? msg[lo] : (lo == NWORDS ? 0x80u : 0u);
        const uint32_t wh = hi < NWORDS ? msg[hi] : (hi == NWORDS ? 0x80u : 0u);
        w[i] = be64_from_le32(wl, wh);
    }
    w[15] = (uint64_t)NWORDS * 32u;   // bit length (len < 2^61)
    uint64_t st[8];
    sha512_init(st);
    sha512_compress(st, w);
    sha512_digest_le32(out, st);
}

}  // namespace nw
