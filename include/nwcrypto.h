/*
 * nwcrypto — MI355X-native Ed25519 verification and SHA-512 digesting for Narwhal/Bullshark.
 *
 * C ABI drop-in boundary for the reference ``crypto`` crate's hot path.
 * Every entry point names the reference interface it replaces.  All buffers are caller-owned;
 * calls are synchronous unless the name ends in ``_dev`` (those enqueue on a caller stream and
 * take device pointers).  There is no CPU fallback: with no usable GPU every call returns
 * NW_ERR_DEVICE.
 *
 * Threading (the worker calls verify_batch from 64 rayon threads, worker/src/processor.rs:75-79):
 * a context is reentrant.  Each call leases its own stream and scratch from a pool (up to 64
 * concurrent calls; more wait), so calls from different threads run concurrently on the GPU.  The
 * key cache is read-shared by verify calls; nw_committee_load takes it exclusively and waits for
 * in-flight calls first.  A ``_dev`` call's scratch stays reserved until its work completes on the
 * caller's stream.  nw_last_error() reports the calling thread's last error.
 *
 * Batch coefficients: every batch entry point takes ``zseed``, which MUST be 32 fresh CSPRNG bytes
 * per call in production (the reference draws z_i from thread_rng on every call).  With a fixed or
 * public seed an attacker can build invalid signatures whose batch terms cancel.  NULL is rejected
 * with NW_ERR_ARG.
 *
 * Verdict semantics are those of ed25519-dalek 1.0.1 (default features + "batch"):
 *   strict  = crypto::Signature::verify      (crypto/src/lib.rs:200-204) -> verify_strict
 *   batch   = crypto::Signature::verify_batch (crypto/src/lib.rs:206-219) -> dalek::verify_batch,
 *             with the random 128-bit coefficients drawn from a seeded ChaCha20 stream
 *             (NW-Z v1, see nw_chacha.h) instead of thread_rng.
 */
#ifndef NWCRYPTO_H
#define NWCRYPTO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes.  NW_ERR_SIG is the reference's opaque ``ed25519::Error`` (CryptoError,
 * crypto/src/lib.rs:18) that callers map to DagError::InvalidSignature (primary/src/error.rs:27-28). */
#define NW_OK 0
#define NW_ERR_SIG 1
#define NW_ERR_ARG 2
#define NW_ERR_DEVICE 3
#define NW_ERR_NOMEM 4

/* ABI revision of this header.  2: nw_verify_certs_dev gained ``d_status`` before ``stream`` and
 * every batch entry point rejects a NULL zseed (revision 1 = nwcrypto 0.1).  The shared library's
 * soname carries it (libnwcrypto.so.2), so a caller built against revision 1 does not load this
 * library by accident; callers may also compare nw_abi_version() with NW_ABI_VERSION at startup. */
#define NW_ABI_VERSION 2

/* Per-signature flag bits written by the verify kernels (nw_verify_certs sig_flags output). */
#define NW_F_S_OK 0x001u      /* S < l (ed25519 high-bit check + dalek check_scalar) */
#define NW_F_A_OK 0x002u      /* public key decodes (dalek::PublicKey::from_bytes) */
#define NW_F_MATCH 0x004u     /* R decodes and R == sB - hA (strict equation holds) */
#define NW_F_STRICT 0x008u    /* verify_strict verdict */
#define NW_F_A_SMALL 0x010u   /* A is of small order */
#define NW_F_R_SMALL 0x020u   /* R is of small order (meaningful when MATCH) */
#define NW_F_SLOW 0x1000u     /* needed the exact batch equation (rare path) */
#define NW_F_R_BAD 0x2000u    /* R failed to decode (found on the exact path) */
/* Bits 0x4000 and above (other than the torsion coefficient at 0x700) are reserved: never set in
 * returned flags.  A signature inside no certificate's vote range gets flags 0 (no verdict). */

/* Opaque extended-point encoding exchanged between shards of one split batch
 * (nw_verify_batch_partial / nw_points_sum_is_identity): 160 bytes. */
#define NW_POINT_BYTES 160

typedef struct nw_ctx nw_ctx;

/* nw_opts.flags */
#define NW_OPT_NO_KEY_NEGTAB 0x1u     /* never store the key tables' negated copies (half the HBM per key;
                                         k_verify's key pass then negates entries in the addition) */

typedef struct nw_opts {
    int device;        /* HIP device ordinal (one process per GPU; -1 = current device) */
    uint32_t flags;    /* NW_OPT_* bits below; other bits are reserved (NW_ERR_ARG) */
    size_t max_keys;   /* key-cache capacity in keys.  0 = as many as the key budget holds.  The key
                          budget is the HBM free on the device at the first nw_committee_load (after
                          this context's basepoint table and anything other contexts or processes
                          hold) less a workspace reserve of max(16 GiB, 1/16 of HBM): ~258 GB on an
                          otherwise idle MI355X.  In committee mode (key_window -1) a non-zero
                          max_keys declares every key the context will ever load: the window is sized
                          for max_keys keys and the first load allocates all of them at once (the
                          worker's two Processors: max_keys = 200,000, two loads of 100,000). */
    int key_window;    /* key comb window: 8, 9, 12, 13, 16 or 20 bits.  0 = auto at the first load (16
                          for <= 384 keys, 12 for <= 12288 keys, else 8); -1 = committee mode: the
                          widest window whose tables fit the key budget is used, for max_keys keys
                          when set, else for the first load's keys with 25% headroom (on an idle
                          MI355X: W20 up to ~236 keys, W16 up to ~3,000, W13 up to ~19,600: a
                          10,000-validator committee; W9 up to ~216,000: the worker's 100,000 keys,
                          or its 200,000 declared through max_keys).  Table bytes per key: w8 0.53 MB,
                          w9 0.95 MB, w12 5.77 MB, w13 10.5 MB, w16 67.1 MB, w20 872 MB; additions per
                          signature 32 / 29 / 22 / 20 / 16 / 13; twice the bytes when the tables
                          carry their negated copies (nw_key_negtab).  (The basepoint comb is fixed
                          at w24: 11 additions, 11.8 GB, shared by every context of the process on
                          the same device.) */
} nw_opts;

/* One certificate: its votes are sig[first_vote .. first_vote + n_votes). */
typedef struct nw_cert {
    uint32_t first_vote;
    uint32_t n_votes;
} nw_cert;

/* ---- context ------------------------------------------------------------------------------- */
int nw_ctx_create(nw_ctx** out, const nw_opts* opts);
void nw_ctx_destroy(nw_ctx* ctx);
/* Human-readable description of the calling thread's last error. */
const char* nw_last_error(const nw_ctx* ctx);

/* ---- committee / key cache -------------------------------------------------------------------
 * Replaces the per-vote ``dalek::PublicKey::from_bytes`` decompression at crypto/src/lib.rs:216
 * (and :202) with a one-time decompression + fixed-base table build per key.  A key that fails
 * to decode is still cached with its failure recorded, so verification returns NW_ERR_SIG for it
 * exactly where the reference's ``?`` would.  Returns the slot index of each key in ``slot_out``
 * (may be NULL).  Keys already cached keep their slot. ``stake`` may be NULL (stake 0). */
int nw_committee_load(nw_ctx* ctx, const uint8_t (*pk)[32], const uint32_t* stake, size_t n,
                      uint32_t* slot_out);
/* Number of cached keys. */
size_t nw_committee_size(const nw_ctx* ctx);
/* Key comb window in use (8 / 12 / 16 / 20; 0 before the first load, or -1 while committee mode
 * has not sized it yet). */
int nw_key_window(const nw_ctx* ctx);
/* 1 when every cached key table is stored with its negated copy (decided at the first load: when
 * twice the tables fit the HBM budget of a committee-mode, declared-size (nw_opts.max_keys) or
 * explicit-window context; never with an automatic window; the flag NW_OPT_NO_KEY_NEGTAB in
 * nw_opts.flags disables it), else 0.  Verdicts are the
 * same either way; only k_verify's key pass differs (no conditional negation with the copies). */
int nw_key_negtab(const nw_ctx* ctx);
/* Basepoint comb window this library was built with (additions per s*B = ceil(256 / w)). */
int nw_base_window(void);

/* ---- verification ----------------------------------------------------------------------------
 * Keys: nw_verify_strict[_many] and nw_verify_batch accept ANY key, like the reference (which
 * decompresses every key per call, crypto/src/lib.rs:202,216).  When every key of a call is in the
 * key cache the call uses the cached comb tables; otherwise it runs the variable-base path (strict:
 * per-signature decompression + windowed scalar multiplication; batch: a Pippenger multi-scalar
 * multiplication) and leaves the cache unchanged.  Verdicts are identical on both paths.
 *
 * crypto::Signature::verify (crypto/src/lib.rs:200-204): strict single verify of ``msg``. */
int nw_verify_strict(nw_ctx* ctx, const uint8_t* msg, size_t len, const uint8_t pk[32],
                     const uint8_t sig[64]);

/* Bulk strict verify (Header::verify / Vote::verify callers, primary/src/messages.rs:48-67,131-142):
 * n independent (msg_i, pk_i, sig_i); ok[i] = 1 when verify_strict accepts. */
int nw_verify_strict_many(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len,
                          const uint8_t (*pk)[32], const uint8_t (*sig)[64], size_t n, uint8_t* ok);

/* dalek::verify_batch as called by crypto::Signature::verify_batch (crypto/src/lib.rs:218) and by
 * the worker's simulated load (worker/src/processor.rs:78): one verdict for n signatures over
 * per-signature messages.  Coefficients: NW-Z v1 stream ``zseed`` with batch index ``batch_index``.
 * Returns NW_OK / NW_ERR_SIG. */
int nw_verify_batch(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len,
                    const uint8_t (*pk)[32], const uint8_t (*sig)[64], size_t n,
                    const uint8_t zseed[32], uint64_t batch_index);

/* Many dalek::verify_batch calls over arbitrary keys in one submission (the worker's direct call,
 * worker/src/processor.rs:78, without a key cache): batch b is the next counts[b] signatures;
 * batch_ok[b] = 1 iff its batch equation holds (coefficients: NW-Z v1 with batch index
 * batch_base + b).  Always the variable-base Pippenger path. */
int nw_verify_batches_pk(nw_ctx* ctx, size_t nb, const uint32_t* counts, const uint8_t* const* msg,
                         const size_t* len, const uint8_t (*pk)[32], const uint8_t (*sig)[64],
                         const uint8_t zseed[32], uint64_t batch_base, uint8_t* batch_ok);

/* One shard of a batch split across GPUs: the shard's share of the batch
 * equation, sum z_i R_i + sum (z_i h_i mod l) A_i - (sum z_i s_i mod l) B over its n signatures,
 * with z_i drawn at coefficient index z_offset + i of batch ``batch_index``.  ``point`` receives the
 * sum (NW_POINT_BYTES, opaque); *bad = 1 when a signature fails to parse or decode (the batch is
 * then Err).  The batch verdict is Ok iff no shard is bad and nw_points_sum_is_identity of all
 * shards' points is true. */
int nw_verify_batch_partial(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len,
                            const uint8_t (*pk)[32], const uint8_t (*sig)[64], size_t n,
                            const uint8_t zseed[32], uint64_t batch_index, uint32_t z_offset,
                            uint8_t point[NW_POINT_BYTES], int* bad);
int nw_points_sum_is_identity(nw_ctx* ctx, const uint8_t (*points)[NW_POINT_BYTES], size_t k,
                              int* is_identity);

/* Certificate bulk path (Certificate::verify's batch step, primary/src/messages.rs:214, for many
 * certificates at once).  Signers are committee slots (nw_committee_load).  msg[c] is the 32-byte
 * certificate digest.  Vote ranges must be pairwise disjoint (a vote's coefficient and exact-path
 * term belong to one certificate): overlapping ranges are NW_ERR_ARG; a signature inside no range
 * gets sig_ok 0 and affects no certificate.  Outputs (each may be NULL):
 *   cert_ok[c]        1 iff Signature::verify_batch(msg[c], votes of c) is Ok
 *   sig_ok[v]         1 iff verify_strict accepts vote v (the per-signature fallback bitmap)
 *   accepted_stake[c] sum of signer stake over votes with sig_ok = 1
 * Coefficients for certificate c use batch index cert_base + c. */
int nw_verify_certs(nw_ctx* ctx, const nw_cert* certs, size_t ncerts, const uint8_t (*sig)[64],
                    const uint32_t* signer_slot, const uint8_t (*msg)[32], const uint8_t zseed[32],
                    uint64_t cert_base, uint8_t* cert_ok, uint8_t* sig_ok, uint64_t* accepted_stake);

/* Many independent dalek::verify_batch calls in one submission — the worker's simulated
 * transaction-signature load (worker/src/processor.rs:75-79: 64 chunks per batch, 8-byte messages,
 * keys fixed at spawn).  Batch b covers signatures [first[b], first[b] + n[b]); signature i signs
 * msg[i] (len[i] bytes) under key-cache slot signer_slot[i] (nw_committee_load).  Outputs (each
 * may be NULL): batch_ok[b] = 1 iff verify_batch of batch b is Ok (coefficients: NW-Z v1 with
 * batch index batch_base + b); sig_ok[i] = verify_strict verdict of signature i. */
int nw_verify_batches(nw_ctx* ctx, size_t nb, const uint32_t* first, const uint32_t* n,
                      const uint8_t* const* msg, const size_t* len, const uint32_t* signer_slot,
                      const uint8_t (*sig)[64], const uint8_t zseed[32], uint64_t batch_base, uint8_t* batch_ok,
                      uint8_t* sig_ok);

/* Device-resident variant for streaming use (inputs already in HBM).  All pointers are device
 * pointers; ``stream`` is a hipStream_t (NULL = default stream).  ``sig_flags`` (uint32 per vote,
 * NW_F_* bits) may be NULL.  The inputs are checked on the device (every vote range inside
 * [0, nsigs), no vote inside two ranges, every signer slot inside the key cache); the kernels clamp
 * them, so bad inputs never fault — their signatures and certificates are rejected.
 *   d_status == NULL: the check is synchronous — the call waits for it on ``stream`` and returns
 *                     NW_ERR_ARG (enqueueing nothing else) when it fails; otherwise it enqueues the
 *                     verification and returns.
 *   d_status != NULL: fully asynchronous — *d_status (device uint32) receives NW_OK or NW_ERR_ARG
 *                     in stream order. */
int nw_verify_certs_dev(nw_ctx* ctx, size_t ncerts, const uint32_t* d_cert_first,
                        const uint32_t* d_cert_nvotes, size_t nsigs, const uint8_t* d_sig64,
                        const uint32_t* d_signer_slot, const uint8_t* d_msg32,
                        const uint8_t zseed[32], uint64_t cert_base, uint8_t* d_cert_ok,
                        uint32_t* d_sig_flags, uint64_t* d_accepted_stake, uint32_t* d_status,
                        void* stream);

/* ---- digests ---------------------------------------------------------------------------------
 * sha2 0.9 Sha512 via ed25519_dalek::Sha512 (primary/src/messages.rs:72-82,147-151,228-232;
 * worker/src/processor.rs:65; worker/src/batch_maker.rs:125).  Callers truncate to 32 bytes. */
int nw_sha512(nw_ctx* ctx, const uint8_t* data, size_t len, uint8_t out[64]);
int nw_sha512_many(nw_ctx* ctx, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                   size_t n, uint8_t (*out)[64]);
/* Device-resident bulk digest: d_base/d_off/d_len/d_out are device pointers.  Each message is one
 * sequential compression chain: a lone 508,052-B worker batch takes ~12-15 ms whatever the number
 * of batches in the call (up to ~1,000 chains run concurrently at that rate), DESIGN.md §5.5. */
int nw_sha512_many_dev(nw_ctx* ctx, const uint8_t* d_base, const uint64_t* d_off,
                       const uint64_t* d_len, size_t n, uint8_t* d_out64, void* stream);

/* Asynchronous many-message digest from host buffers, for a caller that keeps receiving work while
 * the GPU hashes (the worker's Processor loop, worker/src/processor.rs:63-97, replacing one
 * serial Sha512::digest per batch at :65 by one submission per window of batches).  Message i is
 * msg[i] (len[i] bytes); the buffers must stay valid until nw_job_wait returns (the worker keeps
 * each batch until it is stored under its digest anyway).  The call enqueues the upload, the
 * digest kernel and the download and returns a job at once.
 *   nw_job_done(job): 1 when the digests are ready, 0 while in flight, < 0 on a device error.
 *   nw_job_wait(job): blocks until out (n x 64 bytes) holds the digests, then frees the job; every
 *                     job must be waited for exactly once, before nw_ctx_destroy.
 * A job holds one of the context's 64 call workspaces until it is waited for; at most 32 jobs may be
 * unwaited at once (the rest of the pool stays for synchronous calls): a 33rd submit returns
 * NW_ERR_NOMEM at once rather than blocking. */
typedef struct nw_job nw_job;
int nw_sha512_many_async(nw_ctx* ctx, const uint8_t* const* msg, const size_t* len, size_t n,
                         uint8_t (*out)[64], nw_job** job);
int nw_job_done(nw_job* job);
int nw_job_wait(nw_job* job);

/* ---- signing (crypto::Signature::new / generate_keypair, crypto/src/lib.rs:163-191) -------------
 * Low-volume in the reference; here it makes synthetic workloads.  RFC 8032 Ed25519 over
 * messages of exactly ``msg_len`` bytes (8 or 32). pk or sig may be NULL. */
int nw_sign_many(nw_ctx* ctx, const uint8_t (*seed)[32], const uint8_t* msgs, size_t msg_len,
                 size_t n, uint8_t (*pk)[32], uint8_t (*sig)[64]);
int nw_sign_many_dev(nw_ctx* ctx, const uint8_t* d_seed32, const uint8_t* d_msgs, size_t msg_len,
                     size_t n, uint8_t* d_pk32, uint8_t* d_sig64, void* stream);

/* ---- measurement --------------------------------------------------------------------------
 * When enabled, HIP events are recorded on the launch stream around every k_verify launch; read
 * back (synchronizing those events) the summed device time and launch count, then reset.  Launches
 * of at most 4,096 signatures run k_verify_split with k_finish's work fused into it (no separate
 * k_finish launch): their samples cover verify + finish, so they are not comparable with large
 * launches' samples (k_verify alone) or with builds before that fusion. */
int nw_profile_enable(nw_ctx* ctx, int on);
int nw_profile_read(nw_ctx* ctx, double* verify_ms_total, uint64_t* verify_launches);
/* Same, plus the signatures covered by those launches (the roofline's work per launch). */
int nw_profile_read_sigs(nw_ctx* ctx, double* verify_ms_total, uint64_t* verify_launches,
                         uint64_t* verify_sigs);

/* ---- primary certificate path -------------------------------------
 * Native ingestion of bincode ``PrimaryMessage`` frames (primary/src/primary.rs:236) and the whole
 * of Certificate::verify (primary/src/messages.rs:189-215, Header::verify :48-67) for many
 * certificates: host checks in C++, all crypto on the GPU in three submissions.  Verdicts are the
 * DagError kinds the reference returns (primary/src/error.rs:24-58), checked in its order. */
#define NW_DAG_PENDING (-1)             /* decode only: needs the GPU checks */
#define NW_DAG_OK 0
#define NW_DAG_INVALID_SIGNATURE 1      /* DagError::InvalidSignature */
#define NW_DAG_SERIALIZATION 2          /* DagError::SerializationError (bincode / base64 key) */
#define NW_DAG_INVALID_HEADER_ID 3      /* DagError::InvalidHeaderId */
#define NW_DAG_MALFORMED_HEADER 4       /* DagError::MalformedHeader */
#define NW_DAG_UNKNOWN_AUTHORITY 5      /* DagError::UnknownAuthority */
#define NW_DAG_AUTHORITY_REUSE 6        /* DagError::AuthorityReuse */
#define NW_DAG_REQUIRES_QUORUM 7        /* DagError::CertificateRequiresQuorum */
#define NW_DAG_NOT_CERTIFICATE 8        /* a valid PrimaryMessage variant other than Certificate */

/* Committee (config/src/lib.rs:161-240): authority i is name[i] with stake[i]; its worker ids are
 * worker_id[worker_first[i] .. worker_first[i + 1]) (worker_first has n + 1 entries; both NULL =
 * no workers, so any header with a payload is MalformedHeader). */
typedef struct nw_committee {
    size_t n;
    const uint8_t (*name)[32];
    const uint32_t* stake;
    const uint32_t* worker_first;
    const uint32_t* worker_id;
} nw_committee;

typedef struct nw_cert_batch nw_cert_batch;

/* Decoded view of one certificate of a batch.  Pointers stay valid until nw_cert_batch_free. */
typedef struct nw_cert_view {
    int32_t status;                  /* NW_DAG_PENDING, or a final verdict found while decoding
                                        (SERIALIZATION, NOT_CERTIFICATE, OK for genesis) */
    int32_t header_error;            /* Header::verify check after the id (UNKNOWN_AUTHORITY /
                                        MALFORMED_HEADER) or NW_DAG_OK */
    int32_t quorum_error;            /* quorum check (AUTHORITY_REUSE / UNKNOWN_AUTHORITY /
                                        REQUIRES_QUORUM) or NW_DAG_OK */
    uint64_t round;
    const uint8_t* author;           /* 32 B */
    const uint8_t* header_id;        /* 32 B */
    const uint8_t* header_sig;       /* 64 B */
    const uint8_t* header_preimage;  /* Hash for Header (primary/src/messages.rs:70-84) */
    size_t header_preimage_len;
    const uint8_t* cert_preimage;    /* 72 B: Hash for Certificate (:226-234) */
    uint32_t first_vote, n_votes;
    const uint8_t* vote_keys;        /* [n_votes][32] */
    const uint8_t* vote_sigs;        /* [n_votes][64] */
} nw_cert_view;

/* Host only (no context, no GPU): decode n frames and run the host-side checks. */
int nw_cert_batch_decode(const nw_committee* committee, const uint8_t* const* frame, const size_t* len,
                         size_t n, nw_cert_batch** out);
size_t nw_cert_batch_size(const nw_cert_batch* batch);
int nw_cert_batch_view(const nw_cert_batch* batch, size_t i, nw_cert_view* out);
void nw_cert_batch_free(nw_cert_batch* batch);
/* The GPU half: header/certificate digests, header signatures, vote batches.  verdict[i] receives
 * the NW_DAG_* verdict of certificate i.  Batch coefficients (NW-Z v1) use batch index cert_base + j
 * for the j-th certificate that reaches the batch step. */
int nw_cert_batch_verify(nw_ctx* ctx, const nw_cert_batch* batch, const uint8_t zseed[32],
                         uint64_t cert_base, int32_t* verdict);
/* decode + verify + free in one call. */
int nw_certificates_verify(nw_ctx* ctx, const nw_committee* committee, const uint8_t* const* frame,
                           const size_t* len, size_t n, const uint8_t zseed[32], uint64_t cert_base,
                           int32_t* verdict);

/* Library build identifier (gfx target, build date). */
const char* nw_version(void);
/* NW_ABI_VERSION the library was built with. */
int nw_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NWCRYPTO_H */
