// Two-lane SHA-512 compression: one message on a lane pair, for the latency of a lone chain (a
// 6,667-parent header, the worker batches when only a few are in flight).
//
// A lone wave issues one VALU instruction per ~4-5 cycles whatever its active lanes, so a chain's
// time is its instruction count.  The 80 rounds carry two recurrences (FIPS 180-4 §6.4.2, with
// d_t = a_{t-3}, h_t = e_{t-3}):
//     e_{t+1} = a_{t-3} + t1_t,   t1_t = e_{t-3} + K_t + W_t + Sigma1(e_t) + Ch(e_t, e_{t-1}, e_{t-2})
//     a_{t+1} = t1_t + t2_t,      t2_t = Sigma0(a_t) + Maj(a_t, a_{t-1}, a_{t-2})
// The even lane of a pair runs the e-chain, the odd lane the a-chain TWO ROUNDS BEHIND: at step t
// the even lane holds (e_t, e_{t-1}, e_{t-2}, e_{t-3}) and produces e_{t+1}; the odd lane holds
// (a_{t-2}, a_{t-3}, a_{t-4}, a_{t-5}) and produces a_{t-1} = t2_{t-2} + t1_{t-2}, where
// t1_{t-2} = e_{t-1} - a_{t-5}.  With that skew each lane needs exactly the partner's SECOND newest
// value (e_{t-1} resp. a_{t-3} = d_t), so one step is the same 20 instructions on both lanes:
//     S = Sigma(x0)            per-lane rotations: Sigma1(x) = rotr14(x ^ rotr4(x) ^ rotr27(x)),
//                              Sigma0(x) = rotr28(x ^ rotr6(x) ^ rotr11(x))      8 (6 alignbit, 2 bitop3)
//     F = Ch(x0 ^ (m & ~x1), x1, x2)    = Ch on the even lane, Maj on the odd one  4 (bitop3)
//     Z = (x3 ^ m) + kw        = h + K_t + W_t (even, kw = K_t + W_t) / -a_{t-5} (odd, kw = 1)  3
//     new = S + F + Z + swap(x1)   swap = DPP quad_perm [1,0,3,2] of a value 2 steps old  5
// against 27 per round on one lane, and the exchanged value is never on the critical path (no DPP
// wait states).  A block is 82 steps: the odd lane's first two outputs (a_{-1}, a_0) are the known
// b, a, and the even lane idles through the last two.  Each lane feeds forward only its own half
// of the chaining state (even: e f g h, odd: a b c d).
#pragma once
#include "nw_sha512.h"

namespace nw {

NW_HD uint64_t rotr64v(uint64_t x, uint32_t n) {   // 0 < n < 32, per lane
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    uint64_t r = ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
    asm("" : "+v"(r));   // opaque (see bitop3_64): one v_lshl_add_u64 per later 64-bit add
    return r;
#else
    return __builtin_rotateright64(x, n);
#endif
}

// value of the partner lane (lane ^ 1); device only.  (Reading it through the add itself,
// v_add_co/v_addc_co _dpp, saves the two moves but leaves the bitop3 results without the
// independent instructions that cover their wait states: the compiler then pads with s_nop.)
__device__ __forceinline__ uint64_t swap_pair64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, 0xB1, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), 0xB1, 0xF, 0xF, false);
    uint64_t r = ((uint64_t)hi << 32) | lo;
    asm("" : "+v"(r));
    return r;
#else
    return x;
#endif
}

NW_HD uint64_t sel64(uint64_t m, uint64_t a, uint64_t b) { return bitop3_64<0xCA>(m, a, b); }   // m ? a : b

struct Sha2L {
    uint64_t m;              // 0 on the even lane (e-chain), ~0 on the odd lane (a-chain)
    uint32_t rp, rq, rr;     // Sigma rotation amounts of this lane's chain

    __device__ __forceinline__ void init(bool odd) {
        m = odd ? ~0ull : 0ull;
        rp = odd ? 6u : 4u;
        rq = odd ? 11u : 27u;
        rr = odd ? 28u : 14u;
    }

    // one step: (A, B, C, D) = own values newest first; returns the new value (replaces D)
    __device__ __forceinline__ uint64_t step(uint64_t A, uint64_t B, uint64_t C, uint64_t D, uint64_t kw) const {
        const uint64_t s = rotr64v(xor3_64(A, rotr64v(A, rp), rotr64v(A, rq)), rr);
        const uint64_t f = bitop3_64<0xCA>(bitop3_64<0xD2>(A, B, m), B, C);
        const uint64_t z = (D ^ m) + kw;
        return s + (f + (z + swap_pair64(B)));
    }

    // K_t + W_t is read KW_AHEAD steps before its use into a register ring: a read issued in the
    // step that consumes it exposes the whole LDS latency (~50-120 cycles on a 20-instruction step)
    // to the chain once per round.  PAIRED: kw(t) for even t returns (K_t + W_t, K_{t+1} + W_{t+1})
    // from one 128-bit LDS read, refilling two ring slots every other step (half the reads; the ring
    // holds two more entries so a refill never overwrites a value not yet consumed).
    static constexpr int KW_AHEAD = 4;
    static_assert(KW_AHEAD % 2 == 0, "paired reads start on even rounds");
    template <bool PAIRED>
    static constexpr int ring() { return PAIRED ? KW_AHEAD + 2 : KW_AHEAD; }

    // step T of a block on the register array x (the roles rotate with period 4; T is a
    // compile-time constant so every index below is a fixed register)
    template <int T, bool PAIRED, class KW>
    __device__ __forceinline__ void block_step(uint64_t x[4], const uint64_t h[4], uint64_t* q, KW& kw) const {
        constexpr int RING = ring<PAIRED>();
        uint64_t& D = x[(7 - T) & 3];
        // steps 80, 81: the even lane's result is discarded, the odd lane's kw must still be 1:
        // they reuse K_79 + W_79's slot, which is never refilled
        const uint64_t k = q[(T < 80 ? T : 79) % RING];
        if constexpr (PAIRED) {
            if constexpr ((T & 1) == 0 && T + KW_AHEAD < 80) {
                const auto pr = kw(T + KW_AHEAD);
                q[(T + KW_AHEAD) % RING] = pr.x;
                q[(T + KW_AHEAD + 1) % RING] = pr.y;
            }
        } else {
            if constexpr (T + KW_AHEAD < 80) q[T % RING] = kw(T + KW_AHEAD);
        }
        uint64_t nv = step(x[(4 - T) & 3], x[(5 - T) & 3], x[(6 - T) & 3], D, k);
        if (T == 0) nv = sel64(m, h[1], nv);           // odd: a_{-1} = b
        else if (T == 1) nv = sel64(m, h[0], nv);      // odd: a_0 = a
        else if (T >= 80) nv = sel64(m, nv, D);        // even: keep e..h
        D = nv;
        if constexpr (T + 1 < 82) block_step<T + 1, PAIRED>(x, h, q, kw);
    }

    // One compression.  h = this lane's half of the chaining state (even: e f g h, odd: a b c d);
    // kw(t) = K_t + W_t on the even lane and 1 on the odd lane, t = 0..79 (PAIRED: rounds t, t + 1
    // for even t, as a ulonglong2).
    template <bool PAIRED = false, class KW>
    __device__ __forceinline__ void block(uint64_t h[4], KW kw) const {
        uint64_t q[ring<PAIRED>()];
        if constexpr (PAIRED) {
#pragma unroll
            for (int t = 0; t < KW_AHEAD; t += 2) {
                const auto pr = kw(t);
                q[t] = pr.x;
                q[t + 1] = pr.y;
            }
        } else {
#pragma unroll
            for (int t = 0; t < KW_AHEAD; ++t) q[t] = kw(t);
        }
        uint64_t x[4];
        x[0] = sel64(m, h[2], h[0]);   // newest: e (even) / a_{-2} = c (odd)
        x[1] = sel64(m, h[3], h[1]);   // f / a_{-3} = d
        x[2] = h[2];                   // g / (unused)
        x[3] = h[3];                   // h / (unused)
        block_step<0, PAIRED>(x, h, q, kw);
        // even: (e f g h) = x[0] x[1] x[2] x[3];  odd: (a b c d) = x[2] x[3] x[0] x[1]
        h[0] += sel64(m, x[2], x[0]);
        h[1] += sel64(m, x[3], x[1]);
        h[2] += sel64(m, x[0], x[2]);
        h[3] += sel64(m, x[1], x[3]);
    }
};

}  // namespace nw
