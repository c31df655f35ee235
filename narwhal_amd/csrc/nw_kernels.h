// Kernel parameter blocks and launchers shared by nw_kernels.hip and the C-ABI host layer.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "../../include/nwcrypto.h"

namespace nw {

// key_info bits (per cached key)
static constexpr uint32_t KI_OK = 1u;             // decodes (dalek::PublicKey::from_bytes ok)
static constexpr uint32_t KI_SMALL = 2u;          // small order
static constexpr uint32_t KI_TORSION_SHIFT = 4;   // 3 bits: t with A^t = t * T8
static constexpr uint32_t NW_F_TCOEF_SHIFT = 8;   // 3 bits of per-signature torsion coefficient
// Exact-path record of a signature whose strict equation fails (k_slow_prep / k_slow_mul /
// k_cert_finalize): an extended point (D_i = R_i - P_i, or z_i D_i once multiplied), its kind, and
// z_i mod 8.
static constexpr int SLOW_WORDS = 44;
static constexpr int SLOW_KIND = 40;              // word: SK_*
static constexpr uint32_t SK_SKIP = 0;            // certificate already rejected: no point computed
static constexpr uint32_t SK_SMALL = 1;           // D_i of small order (or z_i = 0): record = (z_i mod 8) D_i
static constexpr uint32_t SK_BIG = 2;             // D_i has a prime-order component and z_i != 0
static constexpr uint32_t SK_MUL = 3;             // SK_BIG whose z_i D_i was computed (record holds z_i D_i)
// Per-certificate exact-path state word: the number of SK_BIG entries and two rejection flags.
// CS_DOOM: a vote with bad S / undecodable A (set by k_finish, so final before k_slow_prep, which
// skips such certificates' entries).  CS_RDOOM: a vote whose R failed to decode (set by k_slow_prep
// itself; k_slow_prep does NOT skip on it, so every slow entry of a certificate not doomed by
// k_finish decodes its own R and NW_F_R_BAD is the same on every run; k_slow_mul skips both).
static constexpr uint32_t CS_DOOM = 0x80000000u;
static constexpr uint32_t CS_RDOOM = 0x40000000u;
static constexpr uint32_t CS_BIG_MASK = 0x3FFFFFFFu;
// internal flag bit: k_verify parked P_i (extended) in pslow[i] (its y did not match R's); cleared
// by k_slow_prep before the flags reach the caller (every such signature is on the slow list)
static constexpr uint32_t NW_F_P_SAVED = 0x4000u;
// sig_cert value of a signature inside no certificate's vote range: it gets no verdict (flags 0)
// and never touches any certificate's exact-path state
static constexpr uint32_t NO_CERT = 0xFFFFFFFFu;
static constexpr int PBUF_WORDS = 21;             // per-signature k_verify -> k_finish record (X, Z, flags)
#ifndef NW_FINISH_K
#define NW_FINISH_K 16
#endif
static constexpr int FINISH_K = NW_FINISH_K;      // signatures per lane in the batch-inversion kernel
#ifndef NW_INV_VAR
#define NW_INV_VAR 1   // variable-time safegcd where the lanes' inversions are few (k_finish, fused split)
#endif
// Verify launches of at most this many signatures with one signature per k_finish lane (fk = 1) run
// k_verify_split with k_finish's work fused in (nw_verify_split.h): no k_finish launch.
static constexpr uint32_t SPLIT_FUSE_MAX_SIGS = 4096;
inline bool split_fuses_finish(uint32_t gn, uint32_t fk) { return gn <= SPLIT_FUSE_MAX_SIGS && fk == 1; }

static inline unsigned blocks_for(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

struct VerifyParams {
    uint32_t n;                    // signatures (also the SoA row stride of pbuf / pre)
    uint32_t g0, gn;               // processing-order columns [g0, g0 + gn) handled by this launch
    uint32_t fk;                   // k_finish: signatures per lane (1..FINISH_K)
    uint32_t batch_mode;           // 0: strict flags only; 1: batch bookkeeping (z, slow list)
    const uint8_t* sig;            // [n][64]  R || S
    const uint32_t* signer;        // [n] key-cache slot
    const uint32_t* sig_cert;      // [n] certificate / batch index (local), NO_CERT outside every range
    const uint32_t* cert_first;    // [ncerts] first signature of each certificate
    const uint8_t* cert_msg;       // MSGMODE 0: [ncerts][32]
    const uint8_t* msg_base;       // MSGMODE 1: packed messages
    const uint64_t* msg_off;       // MSGMODE 1: [n]
    const uint64_t* msg_len;       // MSGMODE 1: [n]
    uint64_t cert_base;            // global index of certificate 0 (z stream nonce)
    const uint32_t* keys_raw;      // [K][8] raw key words (as hashed)
    const uint32_t* key_info;      // [K]
    const uint32_t* key_tab;       // [K][key_stride]: T+ (comb_words(key_window)), then T- when key_negtab
    const uint32_t* btab;          // [B_TABLES][comb_words(B_WINDOW)] basepoint comb T+, then T- (B_NEGTAB)
    uint64_t key_stride;           // u32 words per key-cache slot
    uint32_t key_negtab;           // every key table is followed by its negated copy
    uint32_t zseed[8];
    uint32_t* flags;               // [n] NW_F_* bits
    uint32_t* slow_count;          // [1]
    uint32_t* slow_list;           // [n]
    uint32_t* slow_slot;           // [n]
    uint32_t* slow_buf;            // [n][SLOW_WORDS]
    uint32_t* pslow;               // [n][40] P_i of signatures whose y did not match (batch mode; may be null)
    uint32_t* cert_state;          // [ncerts] CS_* exact-path state (batch mode)
    uint8_t* ok_out;               // [n] strict verdict bytes written by k_finish (strict calls; may be null)
    uint32_t* pbuf;                // [PREC_ROWS][n] SoA, processing order: P's X, Z + partial flags
    uint32_t* pre;                 // [10][n] SoA prefix products of Z (k_finish scratch)
    const uint32_t* perm;          // [n] processing order for k_verify (signer-grouped) or null
    const uint2* pinfo;            // [n] with perm: (signer slot, sig_cert) of signature perm[g] at g, so
                                   // k_verify reads them coalesced instead of two scattered 4-B loads
    uint32_t nkeys;                // key-cache slots (signer slots >= nkeys are rejected, never read)
    const uint32_t* sig_keys;      // k_verify_var: [n][8] raw key words of each signature (uncached keys)
};

struct FinalizeParams {
    uint32_t ncerts;
    uint32_t nsigs;                // vote ranges past nsigs reject their certificate
    const uint32_t* cert_first;
    const uint32_t* cert_n;
    const uint32_t* flags;
    const uint32_t* signer;
    const uint32_t* stake;         // [K]
    const uint32_t* sig_cert;      // [nsigs] owner certificate of each vote (NO_CERT: none)
    const uint32_t* slow_slot;
    const uint32_t* slow_buf;
    const uint32_t* cert_state;    // [ncerts] CS_*
    uint8_t* cert_ok;              // [ncerts] (may be null)
    uint64_t* accepted_stake;      // [ncerts] (may be null)
    uint8_t* sig_ok;               // [nsigs] strict verdict bytes (may be null; k_flags_to_ok fused)
    uint32_t* exact_count;         // device counter (zeroed by the preamble) of ...
    uint32_t* exact_list;          // [ncerts] ... certificates whose verdict needs the exact sum (k_cert_exact)
};

hipError_t launch_verify(const VerifyParams& p, int msgmode, int key_window, hipStream_t st);
hipError_t launch_finish(const VerifyParams& p, hipStream_t st);
// Exact path of the batch equation: k_slow_prep (every signature with D_i != O: decode R, D_i,
// small-order test) then k_slow_mul (z_i D_i, only for certificates with two or more SK_BIG
// entries); both read the device slow counter, so honest batches find no work.
hipError_t launch_slow(const VerifyParams& p, int msgmode, int key_window, uint32_t n_upper, hipStream_t st);
hipError_t launch_finalize(const FinalizeParams& p, hipStream_t st);
// Calls of at most TAIL_MAX_CERTS certificates finalize in one wave (k_cert_tail); with at most
// SLOW_TAIL_MAX_SIGS signatures as well, the whole exact path and the finalize run in one workgroup
// (k_slow_tail, launch_slow_tail) instead of launch_slow + launch_finalize.
static constexpr uint32_t TAIL_MAX_CERTS = 16;
static constexpr uint32_t SLOW_TAIL_MAX_SIGS = 256;
inline bool slow_tail_fits(uint64_t ncerts, uint64_t nsigs) {
    return ncerts >= 1 && ncerts <= TAIL_MAX_CERTS && nsigs >= 1 && nsigs <= SLOW_TAIL_MAX_SIGS;
}
hipError_t launch_slow_tail(const VerifyParams& p, const FinalizeParams& f, int msgmode, int key_window, hipStream_t st);
// Batch preamble: reset sig_cert to NO_CERT, zero counts (may be null: no histogram) / the slow
// counter / status (may be null: no input check), expand certificates (a vote claimed by two
// certificates is NW_ERR_ARG), histogram + check signer slots (k_prep_certs, k_expand_count); then
// launch_group_scatter (scan + scatter) when counts were built.
hipError_t launch_prep_expand(uint32_t ncerts, uint32_t nsigs, uint32_t nkeys, const uint32_t* first,
                              const uint32_t* nv, const uint32_t* signer, uint32_t* sig_cert, uint32_t* zero4,
                              uint32_t* counts, uint32_t* status, uint32_t* cert_state, hipStream_t st);
hipError_t launch_group_scatter(uint32_t n, uint32_t nkeys, const uint32_t* signer, const uint32_t* sig_cert,
                                const uint32_t* counts, uint32_t* cursor, uint32_t* perm, uint2* pinfo,
                                hipStream_t st);
hipError_t launch_flags_to_ok(uint32_t n, const uint32_t* flags, uint8_t* ok, hipStream_t st);
// Tables for nk keys at tab + j * stride (u32 words); negtab: each followed by its negated copy
// (stride >= 2 comb_words(window)).
hipError_t launch_key_prep(uint32_t nk, const uint32_t* keys_raw, uint32_t* key_info, uint32_t* bases,
                           uint32_t* tab, size_t stride, bool negtab, int window, hipStream_t st);
hipError_t launch_sha512_many(uint32_t n, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                              uint8_t* out, hipStream_t st);
hipError_t launch_sign(uint32_t n, int msg_words, const uint32_t* seeds, const uint32_t* msgs,
                       const uint32_t* btab, uint32_t* pk, uint32_t* sig, hipStream_t st);

}  // namespace nw
