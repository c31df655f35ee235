// ChaCha20 block function (RFC 8439 §2.3) used as the seeded batch-coefficient generator that
// replaces dalek's merlin transcript + thread_rng (SURVEY.md §2 row ★T5, §7 hard part 2).
//   NW-Z v1:  z_i = LE-u128(ChaCha20(key = zseed, counter = i, nonce = u32le(cert_lo) ||
//                                    u32le(cert_hi) || 0)[0:16])
// (oracle/ed25519_oracle.py batch_coefficients is the reference restatement.)
#pragma once
#include "nw_field.h"

namespace nw {

NW_HD uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define NW_QR(a, b, c, d)                          \
    a += b; d = rotl32(d ^ a, 16);                 \
    c += d; b = rotl32(b ^ c, 12);                 \
    a += b; d = rotl32(d ^ a, 8);                  \
    c += d; b = rotl32(b ^ c, 7)

// First 4 words of the keystream block (all the coefficient generator needs).
NW_HD void chacha20_z(uint32_t z[4], const uint32_t key[8], uint32_t counter, uint32_t n0, uint32_t n1,
                      uint32_t n2) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
    uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
    uint32_t x12 = counter, x13 = n0, x14 = n1, x15 = n2;
#pragma nounroll
    for (int r = 0; r < 10; ++r) {
        NW_QR(x0, x4, x8, x12); NW_QR(x1, x5, x9, x13); NW_QR(x2, x6, x10, x14); NW_QR(x3, x7, x11, x15);
        NW_QR(x0, x5, x10, x15); NW_QR(x1, x6, x11, x12); NW_QR(x2, x7, x8, x13); NW_QR(x3, x4, x9, x14);
    }
    z[0] = x0 + 0x61707865u;
    z[1] = x1 + 0x3320646eu;
    z[2] = x2 + 0x79622d32u;
    z[3] = x3 + 0x6b206574u;
}

#undef NW_QR

}  // namespace nw
