// Variable-base verification for keys that are NOT in the committee key cache:
//   * k_verify_var  — strict verify (crypto::Signature::verify, crypto/src/lib.rs:200-204) with the
//                     key decompressed per signature and h*A by a signed radix-16 window;
//   * k_msm_*       — dalek::verify_batch's randomized batch equation (crypto/src/lib.rs:218,
//                     worker/src/processor.rs:78) as a segmented Pippenger multi-scalar
//                     multiplication: one bucket task (one wave) per (batch, window, chunk), LDS
//                     counting sort of the chunk's digits, balanced run accumulation with
//                     cross-lane merges, and a wave-level bucket reduction over DPP/bpermute
//                     shuffles.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace nw {

static constexpr int MSM_CH = 2048;          // entries per bucket task (LDS sort capacity)
static constexpr int MSM_ENT_WORDS = 32;     // one affine Niels entry (y+x, y-x, 2dxy + pad) = 128 B
static constexpr int MSM_PT_WORDS = 40;      // extended point (X, Y, Z, T)
static constexpr int MSM_ZS_WORDS = 12;      // z_i s_i (128 x 253 bits, unreduced)

inline constexpr int msm_nwin_a(int c) { return (254 + c - 1) / c; }   // a_i = z_i h_i mod l < 2^253
inline constexpr int msm_nwin_r(int c) { return (129 + c - 1) / c; }   // z_i < 2^128

struct MsmTask {
    uint32_t e0, e1;      // entry range [e0, e1) (global entry indices)
    uint32_t win;         // window
    uint32_t out;         // index of this task's window partial in MsmParams::wpart
};

struct MsmParams {
    uint32_t nb, nsig;
    uint32_t c;                    // window bits (7 or 8)
    const uint32_t* bfirst;        // [nb] first signature of batch b (batches are consecutive)
    const uint32_t* bcount;        // [nb]
    const uint32_t* sig_batch;     // [nsig] batch of each signature
    const uint8_t* sig;            // [nsig][64] R || S
    const uint32_t* keys;          // [nsig][8]  raw A words (as hashed)
    const uint8_t* msg_base;       // packed messages
    const uint64_t* msg_off;       // [nsig]
    const uint64_t* msg_len;       // [nsig]
    uint64_t msg_flen;             // UINT64_MAX: msg_off / msg_len; else every message has this length,
                                   // back to back from msg_base (the arrays are not uploaded)
    uint64_t batch_base;           // NW-Z v1 nonce of batch 0
    uint32_t z_off;                // NW-Z v1 counter offset (a shard of one huge batch)
    uint32_t zseed[8];
    uint32_t* ent;                 // [2 nsig][32]  R entries then A entries, per batch
    int16_t* dig;                  // [nwin_a][2 nsig] signed digits, window-major
    uint32_t* zs;                  // [12][nsig] z_i s_i, SoA
    uint32_t* bad;                 // [nb] parse / decode failure of any signature of the batch
    // bucket tasks
    const MsmTask* tasks;
    uint32_t ntasks;
    uint32_t* bkt;                 // [ntasks][B][40] complete bucket sums (global scratch)
    uint32_t* part;                // [ntasks][2][64][40] run partials at lane-slice boundaries
    uint32_t* wpart;               // [ntasks][40] window partial sums
    const uint32_t* wfirst;        // [nb * nwin_a + 1] first window partial of (b, win)
    uint32_t one_task_windows;     // every (b, win) has exactly one task, task index b * nwin_a + win:
                                   // its partial IS the window sum (k_msm_wsum skipped)
    // final
    const uint32_t* btab;          // basepoint comb
    uint8_t* batch_ok;             // [nb] verdicts (may be null)
    uint32_t* point_out;           // [nb][40] partial sums before the identity test (may be null)
};

hipError_t launch_msm(const MsmParams& p, hipStream_t st);
hipError_t launch_msm_points_identity(uint32_t npts, const uint32_t* pts, uint8_t* out, hipStream_t st);
// Strict verify of uncached keys: VerifyParams.sig_keys holds each signature's raw key words.
struct VerifyParams;
hipError_t launch_verify_var(const VerifyParams& p, int msgmode, uint32_t* scratch, hipStream_t st);

}  // namespace nw
