// Bulk SHA-512 digests (worker batches, header / vote / certificate digests): sha2 0.9 Sha512 via
// ed25519_dalek::Sha512 (primary/src/messages.rs:72-82,147-151,228-232; worker/src/processor.rs:65).
//
// A message is one Merkle-Damgard chain: block b+1 needs block b's state, so one message never uses
// more than one instruction stream's worth of VALU per round.  What a lone wave sustains is one
// instruction per ~4 cycles (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), so the latency
// of a long message is its instruction count per block times that.  Two kernels:
//
//  * k_sha512_many  - one lane per message, everything in one wave: the throughput form (enough
//                     messages to give every SIMD several waves).
//  * k_sha512_split2 - few messages (worker batches: 1,250 per GPU at C4, a 6,667-parent header):
//                     the message schedule does not depend on the chaining state, so two schedule
//                     waves of the same workgroup compute K_t + W_t of the next blocks into LDS while
//                     the round wave runs the 80 rounds of block b from LDS, each message on a lane
//                     pair (nw_sha512_2l.h: 20 VALU instructions per round for both halves of the
//                     chain); the waves meet at one barrier per block.
#include <hip/hip_runtime.h>
#include "nw_sha512.h"
#include "nw_sha512_2l.h"
#include "nw_kernels.h"

namespace nw {

// Blocks of the padded message of L bytes (L + 0x80 + 16-byte length, rounded up to 128).
__device__ __forceinline__ uint32_t sha512_nblocks(uint64_t L) { return (uint32_t)((L + 17 + 127) / 128); }

// Block b of the padded message (m, L) as 16 big-endian words.  Fast path: a full block at a
// 4-byte-aligned address (32 dword loads).  Otherwise (the 1-2 padding blocks, or an unaligned
// message): the aligned dwords that hold at least one message byte of the block are loaded (an
// aligned dword holding a valid byte never leaves the message's page, so nothing past the buffer is
// touched), realigned with v_alignbyte, and bytes past the message are masked to the padding.
__device__ __forceinline__ void sha512_load_block(const uint8_t* m, uint64_t L, uint64_t b, uint64_t w[16]) {
    const uint64_t nfull = L / 128;
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(m) + b * 128;
    const uint32_t sh = (uint32_t)(a0 & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a0 - sh);
    if (b < nfull && sh == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = be64_from_le32(q[2 * k], q[2 * k + 1]);
        return;
    }
    const int64_t vrem = (int64_t)L - (int64_t)(b * 128);        // message bytes from this block on
    const int32_t v = vrem <= 0 ? 0 : (vrem >= 128 ? 128 : (int32_t)vrem);
    const bool marker = vrem >= 0 && vrem < 128;                // the 0x80 byte lands in this block
    uint32_t u[33];
    if (v > 0) {   // a padding-only block (v == 0) reads nothing: its q[0] may lie past the message
        const int32_t kmax = (v + (int32_t)sh - 1) >> 2;          // last dword with a valid byte
#pragma unroll
        for (int k = 0; k < 33; ++k) u[k] = q[k < kmax ? k : kmax];
    } else {
#pragma unroll
        for (int k = 0; k < 33; ++k) u[k] = 0u;
    }
    uint32_t x[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const uint32_t t = __builtin_amdgcn_alignbyte(u[j + 1], u[j], sh);   // block bytes 4j .. 4j+3
        const int32_t d = v - 4 * j;                                         // valid bytes in this word
        uint32_t r = d >= 4 ? t : (d <= 0 ? 0u : (t & ((1u << (8 * d)) - 1u)));
        if (marker && d >= 0 && d < 4) r |= 0x80u << (8 * d);
        x[j] = r;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = be64_from_le32(x[2 * k], x[2 * k + 1]);
    if (b + 1 == sha512_nblocks(L)) {
        w[14] = L >> 61;
        w[15] = L << 3;
    }
}

NW_HD void sha512_digest_store(uint8_t* out, const uint64_t st[8]) {
    uint32_t d[16];
    sha512_digest_le32(d, st);
    uint4* o = reinterpret_cast<uint4*>(out);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = make_uint4(d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]);
}

// ------------------------------------------------------------------------------------ one lane per message
// Throughput form: bounded to 128 VGPRs so 4 waves share each SIMD (a lone wave issues one VALU
// instruction per ~4 cycles; several waves per SIMD approach the SIMD's full rate).
__global__ void __launch_bounds__(256, 4) k_sha512_many(uint32_t n, const uint8_t* base, const uint64_t* off,
                                                        const uint64_t* len, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* m = base + off[i];
    const uint64_t L = len[i];
    uint64_t st[8];
    sha512_init(st);
    const uint32_t nb = sha512_nblocks(L);
    for (uint32_t b = 0; b < nb; ++b) {
        uint64_t w[16];
        sha512_load_block(m, L, b, w);
        sha512_compress(st, w);
    }
    sha512_digest_store(out + (size_t)i * 64, st);
}

// ------------------------------------------------------------------------------------ schedule / round split
static constexpr uint32_t SPLIT_MAX_N = 32768;    // above: k_sha512_many (every SIMD has work anyway)
// A digest launch of SHA_EXCLUSIVE_MIN_WG or more workgroups that still fits one per CU
// (225 <= n <= 32 x CUs: C4's 1,250 worker batches, a worker window) reserves unused dynamic LDS so
// that no other kernel's workgroup (k_verify: 24 KB) fits beside it: the chains then run on CUs of
// their own instead of sharing SIMD issue with the verify waves of the same step (LDS per CU:
// 160 KB; the workgroup's own 63,360 B + the pad leaves < 24 KB).  The price: such a workgroup
// needs an EMPTY CU, which a running k_verify (its dispatcher refilling every freed slot) may not
// leave until it drains, so a lone header's digest (one workgroup, latency-critical) stays unpadded.
static constexpr uint32_t SHA_EXCLUSIVE_PAD = 80000;
static constexpr uint32_t SHA_EXCLUSIVE_MIN_WG = 8;

// ------------------------------------------------------------------------------------ two-lane split
// The rounds on lane pairs (nw_sha512_2l.h: 20 instructions per round for one message instead of
// the one-lane form's 27): 32 messages per workgroup; lane pair (2j, 2j+1) of the round wave serves
// message j.
//
// At ~3.1 us per block for the rounds, one schedule wave (~3 us of arithmetic per block plus its
// block loads) would set the pace, so TWO schedule waves alternate blocks, each doing half a block's
// schedule per period (one period = the rounds of one block, closed by a barrier):
//   wave A (even blocks), period p:  p even: rows 0..47 of block p + 2;   p odd: rows 48..79 of block p + 1
//   wave B (odd blocks),  period p:  p even: rows 48..79 of block p + 1;  p odd: rows 0..47 of block p + 2
// Block k lives in buffer k % 3 (written in periods k-2 and k-1, read in period k).  A schedule
// wave keeps its 16-word ring in registers between the halves, and loads its next block's words
// one own-block (two periods) ahead.  K_t + W_t is stored once per message (column j); the odd
// lanes of the round wave read a constant column of 1s (their "kw" turns the oldest value into
// its negation, see nw_sha512_2l.h), written once at the start.
static constexpr uint32_t SPLIT2_MSGS = 32;
static constexpr uint32_t SPLIT2_COLS = SPLIT2_MSGS + 1;   // + the column of 1s
static constexpr int SPLIT2_HALF = 48;                      // rows of the first half (16 loaded + 32 computed)

// One block's K_t + W_t for the 33 columns, with rows t and t + 1 (t even) of a column adjacent: the
// round wave reads two rounds' values with one 128-bit LDS read (40 reads per block, not 80).
struct alignas(16) KwBlock {
    uint64_t v[40][SPLIT2_COLS][2];
    __device__ __forceinline__ uint64_t& at(int t, uint32_t col) { return v[t >> 1][col][t & 1]; }
    __device__ __forceinline__ ulonglong2 pair(int t, uint32_t col) const {   // t even
        return *reinterpret_cast<const ulonglong2*>(&v[t >> 1][col][0]);
    }
};

// Block k's raw dwords, loaded ahead of use when the block is a full aligned one (else nothing).
struct RawBlock {
    uint32_t u[32];
    __device__ __forceinline__ static bool fast(const uint8_t* m, uint64_t L, uint64_t k) {
        return k < L / 128 && (reinterpret_cast<uintptr_t>(m) & 3u) == 0;
    }
    __device__ __forceinline__ void issue(const uint8_t* m, uint64_t L, uint64_t k, uint32_t nb) {
        if (k < nb && fast(m, L, k)) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(m + k * 128);
#pragma unroll
            for (int j = 0; j < 32; ++j) u[j] = q[j];
        }
    }
    __device__ __forceinline__ void words(const uint8_t* m, uint64_t L, uint64_t k, uint64_t w[16]) const {
        if (fast(m, L, k)) {
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = be64_from_le32(u[2 * j], u[2 * j + 1]);
        } else {
            sha512_load_block(m, L, k, w);
        }
    }
};

// Schedule rows [R0, R1) of the block whose first 16 words are in w (the ring advances in place:
// after row t >= 16 is produced, w[t & 15] holds W_t).  Rows 16.. run as 16-row groups in a rolled
// loop: the kernel's code (three waves' worth of it) stays well inside the instruction cache.
template <int R0, int R1>
__device__ __forceinline__ void split2_rows(uint64_t w[16], KwBlock& kwb, uint32_t col) {
    static_assert(R0 % 16 == 0 && R1 % 16 == 0, "16-row groups");
    if (R0 == 0) {
#pragma unroll
        for (int t = 0; t < 16; ++t) kwb.at(t, col) = w[t] + SHA512_K[t];
    }
#pragma nounroll
    for (int g = (R0 < 16 ? 16 : R0); g < R1; g += 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), w15 >> 7);
            const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), w2 >> 6);
            w[i] += s0 + w[(i + 9) & 15] + s1;
            kwb.at(g + i, col) = w[i] + SHA512_K[g + i];
        }
    }
}

// PROBE (tools/sha_lone.hip only): 1 = schedule waves skip their arithmetic, 2 = the round wave
// skips its rounds (both keep every barrier), to time each side alone; 3 = the round wave writes
// its shader cycles and 100 MHz ticks instead of the digest.
template <int PROBE = 0>
__global__ void __launch_bounds__(192) k_sha512_split2(uint32_t n, const uint8_t* base, const uint64_t* off,
                                                       const uint64_t* len, uint8_t* out) {
    __shared__ KwBlock kw[3];                      // 63,360 B: two workgroups per CU
    const uint32_t wave = threadIdx.x >> 6;         // 0: rounds, 1: schedule A, 2: schedule B
    const uint32_t lane = threadIdx.x & 63u;
    const bool odd = lane & 1u;
    // rounds: lane pair (2j, 2j+1) -> message j; schedule: lane j < 32 -> message j
    const uint32_t j = wave == 0 ? lane >> 1 : lane;
    // A workgroup with fewer than 32 messages (a lone header or worker batch) fills its idle lane
    // pairs with duplicate chains of its own messages, so the round wave always runs with a full
    // EXEC mask: with 2 of 64 lanes active the same instruction stream took 9.1-16.7 k cycles per
    // block depending on the CU, with every lane active 8.94-8.97 k on every CU
    // (profiles/r04/sha_lone_r04j.jsonl, x_mode 0 vs 7).  Only the owning lanes write a digest.
    const uint32_t wg_n = min(SPLIT2_MSGS, n - blockIdx.x * SPLIT2_MSGS);   // >= 1: grid = ceil(n / 32)
    const uint32_t jm = j < SPLIT2_MSGS ? j % wg_n : j;
    const uint32_t i = blockIdx.x * SPLIT2_MSGS + jm;
    const bool live = j < SPLIT2_MSGS && i < n;
    const bool owner = live && jm == j;
    const uint64_t L = live ? len[i] : 0;
    const uint8_t* m = base + (live ? off[i] : 0);
    const uint32_t nb = live ? sha512_nblocks(L) : 0u;
    uint32_t nbmax = nb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nbmax = max(nbmax, (uint32_t)__shfl_xor((int)nbmax, o, 64));
    if (wave == 0) {
        // the round wave is the chain's critical path: when it shares a SIMD with a schedule wave, the
        // arbiter should pick it first
        __builtin_amdgcn_s_setprio(3);
        for (uint32_t t = lane; t < 3 * 80; t += 64) kw[t / 80].at(t % 80, SPLIT2_MSGS) = 1ull;
        uint64_t h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = SHA512_IV[(odd ? 0 : 4) + k];
        Sha2L c;
        c.init(odd);
        const uint32_t col = odd ? SPLIT2_MSGS : j;
        __syncthreads();
        uint64_t tc0 = 0, tr0 = 0;
        if (PROBE == 3) {
            tc0 = __builtin_amdgcn_s_memtime();
            tr0 = __builtin_amdgcn_s_memrealtime();
        }
        uint64_t twait = 0;
        for (uint32_t b = 0; b < nbmax; ++b) {
            if (b < nb && PROBE != 2) {
                const KwBlock& kb = kw[b % 3];
                c.block<true>(h, [&](int t) { return kb.pair(t, col); });
            }
            if (PROBE == 3) {
                const uint64_t tb = __builtin_amdgcn_s_memtime();
                __syncthreads();
                twait += __builtin_amdgcn_s_memtime() - tb;
            } else {
                __syncthreads();
            }
        }
        if (PROBE == 3) {   // shader cycles and 100 MHz ticks of the round wave (digest slot of message 0)
            if (lane == 0) {
                reinterpret_cast<uint64_t*>(out)[0] = __builtin_amdgcn_s_memtime() - tc0;
                reinterpret_cast<uint64_t*>(out)[1] = __builtin_amdgcn_s_memrealtime() - tr0;
                reinterpret_cast<uint32_t*>(out)[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
                reinterpret_cast<uint64_t*>(out)[4] = twait;   // cycles waiting at the period barriers
            }
            return;
        }
        if (owner) {
            // odd lane: a b c d = digest bytes 0..31; even lane: e f g h = bytes 32..63
            uint4* o = reinterpret_cast<uint4*>(out + (size_t)i * 64 + (odd ? 0 : 32));
            uint32_t d[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                d[2 * k] = bswap32((uint32_t)(h[k] >> 32));
                d[2 * k + 1] = bswap32((uint32_t)h[k]);
            }
            o[0] = make_uint4(d[0], d[1], d[2], d[3]);
            o[1] = make_uint4(d[4], d[5], d[6], d[7]);
        }
        return;
    }
    // schedule waves: A (wave 1) owns the even blocks, B (wave 2) the odd ones
    const uint32_t par = wave - 1;
    if (PROBE == 3 && lane == 0) reinterpret_cast<uint32_t*>(out)[4 + wave] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    RawBlock rb;
    uint64_t w[16];
    const uint32_t k0 = par;                       // first own block
    if (k0 < nb && PROBE != 1) {
        sha512_load_block(m, L, k0, w);            // synchronous: nothing was issued yet
        rb.issue(m, L, k0 + 2, nb);
        split2_rows<0, SPLIT2_HALF>(w, kw[k0 % 3], j);
        if (par == 0) split2_rows<SPLIT2_HALF, 80>(w, kw[k0 % 3], j);   // block 0 complete before period 0
    }
    __syncthreads();
    for (uint32_t p = 0; p < nbmax; ++p) {
        if ((p & 1u) == par) {
            // first half of own block p + 2
            const uint32_t k = p + 2;
            if (k < nb && PROBE != 1) {
                rb.words(m, L, k, w);
                rb.issue(m, L, k + 2, nb);
                split2_rows<0, SPLIT2_HALF>(w, kw[k % 3], j);
            }
        } else {
            // second half of own block p + 1
            const uint32_t k = p + 1;
            if (k < nb && PROBE != 1) split2_rows<SPLIT2_HALF, 80>(w, kw[k % 3], j);
        }
        __syncthreads();
    }
}

hipError_t launch_sha512_many(uint32_t n, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                              uint8_t* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (n <= SPLIT_MAX_N) {
        const uint32_t blocks = blocks_for(n, SPLIT2_MSGS);
        uint32_t pad = 0;
        {
            static const int cus = [] {
                int dev = 0, c = 0;
                if (hipGetDevice(&dev) != hipSuccess ||
                    hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                    return 0;
                return c;
            }();
            static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sha512_split2<0>),
                                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                                               (int)SHA_EXCLUSIVE_PAD);
            if (attr == hipSuccess && blocks >= SHA_EXCLUSIVE_MIN_WG && blocks <= (uint32_t)cus)
                pad = SHA_EXCLUSIVE_PAD;
        }
        hipLaunchKernelGGL(k_sha512_split2<0>, dim3(blocks), dim3(192), pad, st, n, base, off, len, out);
    } else {
        hipLaunchKernelGGL(k_sha512_many, dim3(blocks_for(n, 256)), dim3(256), 0, st, n, base, off, len, out);
    }
    return hipGetLastError();
}

}  // namespace nw
