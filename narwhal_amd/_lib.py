"""ctypes binding of libnwcrypto.so (include/nwcrypto.h).

The shared library is built in-tree (``narwhal_amd/libnwcrypto.so``, see ``__graft_entry__.build``).
There is deliberately no CPU fallback: a missing library raises ``ImportError`` here, and a
missing/unusable GPU makes every context creation fail with ``DeviceError``.

Processes that also use PyTorch must ``import torch`` BEFORE importing this module: torch bundles
its own HIP runtime with the same soname (libamdhip64.so.7), the first one loaded serves both, and
only the torch-first order gives both of them the GPU (tools/probe_runtime.sh on the MI355X box).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# NWCRYPTO_LIB: alternative build of the same library (A/B kernel experiments, tools/ only)
LIB_PATH = os.environ.get("NWCRYPTO_LIB") or os.path.join(_HERE, "libnwcrypto.so")

NW_OK, NW_ERR_SIG, NW_ERR_ARG, NW_ERR_DEVICE, NW_ERR_NOMEM = 0, 1, 2, 3, 4
F_S_OK, F_A_OK, F_MATCH, F_STRICT, F_A_SMALL, F_R_SMALL = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
F_SLOW, F_R_BAD = 0x1000, 0x2000


class DeviceError(RuntimeError):
    """The GPU path is unavailable or failed (NW_ERR_DEVICE / NW_ERR_NOMEM / NW_ERR_ARG)."""


class NwOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("flags", ctypes.c_uint32), ("max_keys", ctypes.c_size_t),
                ("key_window", ctypes.c_int)]


class NwCert(ctypes.Structure):
    _fields_ = [("first_vote", ctypes.c_uint32), ("n_votes", ctypes.c_uint32)]


class NwCommittee(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("name", ctypes.c_void_p), ("stake", ctypes.c_void_p),
                ("worker_first", ctypes.c_void_p), ("worker_id", ctypes.c_void_p)]


class NwCertView(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("header_error", ctypes.c_int32), ("quorum_error", ctypes.c_int32),
                ("round", ctypes.c_uint64), ("author", ctypes.c_void_p), ("header_id", ctypes.c_void_p),
                ("header_sig", ctypes.c_void_p), ("header_preimage", ctypes.c_void_p),
                ("header_preimage_len", ctypes.c_size_t), ("cert_preimage", ctypes.c_void_p),
                ("first_vote", ctypes.c_uint32), ("n_votes", ctypes.c_uint32), ("vote_keys", ctypes.c_void_p),
                ("vote_sigs", ctypes.c_void_p)]


# NW_DAG_* verdicts (include/nwcrypto.h; primary/src/error.rs DagError kinds)
DAG_PENDING, DAG_OK, DAG_INVALID_SIGNATURE, DAG_SERIALIZATION, DAG_INVALID_HEADER_ID = -1, 0, 1, 2, 3
DAG_MALFORMED_HEADER, DAG_UNKNOWN_AUTHORITY, DAG_AUTHORITY_REUSE, DAG_REQUIRES_QUORUM = 4, 5, 6, 7
DAG_NOT_CERTIFICATE = 8

ABI_VERSION = 2    # NW_ABI_VERSION of include/nwcrypto.h this binding is written against

_OPTIONAL = {"nw_abi_version", "nw_profile_read_sigs", "nw_base_window", "nw_cert_batch_decode", "nw_cert_batch_size",
             "nw_cert_batch_view", "nw_cert_batch_free", "nw_cert_batch_verify", "nw_certificates_verify",
             "nw_sha512_many_async", "nw_job_done", "nw_job_wait"}


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libnwcrypto.so not built (%s); run `python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    P, S, U32, U64, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "nw_ctx_create": (I, [ctypes.POINTER(P), ctypes.POINTER(NwOpts)]),
        "nw_ctx_destroy": (None, [P]),
        "nw_last_error": (ctypes.c_char_p, [P]),
        "nw_committee_load": (I, [P, P, P, S, P]),
        "nw_committee_size": (S, [P]),
        "nw_key_window": (I, [P]),
        "nw_key_negtab": (I, [P]),
        "nw_base_window": (I, []),
        "nw_verify_strict": (I, [P, P, S, P, P]),
        "nw_verify_strict_many": (I, [P, P, P, P, P, S, P]),
        "nw_verify_batch": (I, [P, P, P, P, P, S, P, U64]),
        "nw_verify_certs": (I, [P, P, S, P, P, P, P, U64, P, P, P]),
        "nw_verify_certs_dev": (I, [P, S, P, P, S, P, P, P, P, U64, P, P, P, P, P]),
        "nw_verify_batches_pk": (I, [P, S, P, P, P, P, P, P, U64, P]),
        "nw_verify_batch_partial": (I, [P, P, P, P, P, S, P, U64, U32, P, ctypes.POINTER(I)]),
        "nw_points_sum_is_identity": (I, [P, P, S, ctypes.POINTER(I)]),
        "nw_verify_batches": (I, [P, S, P, P, P, P, P, P, P, U64, P, P]),
        "nw_sha512": (I, [P, P, S, P]),
        "nw_sha512_many": (I, [P, P, P, P, S, P]),
        "nw_sha512_many_dev": (I, [P, P, P, P, S, P, P]),
        "nw_sha512_many_async": (I, [P, P, P, S, P, ctypes.POINTER(P)]),
        "nw_job_done": (I, [P]),
        "nw_job_wait": (I, [P]),
        "nw_sign_many": (I, [P, P, P, S, S, P, P]),
        "nw_sign_many_dev": (I, [P, P, P, S, S, P, P, P]),
        "nw_profile_enable": (I, [P, I]),
        "nw_profile_read": (I, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64)]),
        "nw_profile_read_sigs": (I, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "nw_version": (ctypes.c_char_p, []),
        "nw_abi_version": (I, []),
        "nw_cert_batch_decode": (I, [ctypes.POINTER(NwCommittee), P, P, S, ctypes.POINTER(P)]),
        "nw_cert_batch_size": (S, [P]),
        "nw_cert_batch_view": (I, [P, S, ctypes.POINTER(NwCertView)]),
        "nw_cert_batch_free": (None, [P]),
        "nw_cert_batch_verify": (I, [P, P, P, U64, P]),
        "nw_certificates_verify": (I, [P, ctypes.POINTER(NwCommittee), P, P, S, P, U64, P]),
    }
    for name, (res, args) in sig.items():
        if name in _OPTIONAL and not hasattr(lib, name):
            continue   # older library build loaded for an A/B run (NWCRYPTO_LIB)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if LIB_PATH == os.path.join(_HERE, "libnwcrypto.so"):
        abi = lib.nw_abi_version() if hasattr(lib, "nw_abi_version") else 1
        if abi != ABI_VERSION:
            raise ImportError("libnwcrypto.so has ABI %d, this binding expects %d: rebuild it" % (abi, ABI_VERSION))
    return lib


LIB = _load()


def _buf(b: bytes):
    return ctypes.c_char_p(b) if b else None


POINT_BYTES = 160   # NW_POINT_BYTES


NW_OPT_NO_KEY_NEGTAB = 0x1   # nw_opts.flags (include/nwcrypto.h)


class Engine:
    """One nw_ctx (one GPU).  Thread-safe and reentrant: every call leases its own stream and
    scratch in the C layer, so calls from several threads run concurrently."""

    def __init__(self, device: int = -1, max_keys: int = 0, key_window: int = 0, flags: int = 0):
        self._ctx = ctypes.c_void_p()
        opts = NwOpts(device, flags, max_keys, key_window)
        rc = LIB.nw_ctx_create(ctypes.byref(self._ctx), ctypes.byref(opts))
        if rc != NW_OK:
            raise DeviceError("nw_ctx_create failed (rc=%d): no usable gfx950 GPU" % rc)
        self.device = device

    # -- plumbing -----------------------------------------------------------------------------
    @property
    def handle(self):
        return self._ctx

    def close(self):
        if self._ctx:
            LIB.nw_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, what: str):
        if rc in (NW_OK, NW_ERR_SIG):
            return rc
        err = LIB.nw_last_error(self._ctx)
        raise DeviceError("%s failed (rc=%d): %s" % (what, rc, err.decode() if err else ""))

    # -- key cache ----------------------------------------------------------------------------
    def committee_load(self, pks, stakes=None):
        """Load keys (iterable of 32-byte bytes); returns their slots (list of int)."""
        pks = [bytes(k) for k in pks]
        n = len(pks)
        blob = b"".join(pks)
        slots = (ctypes.c_uint32 * max(n, 1))()
        st = None
        if stakes is not None:
            st = (ctypes.c_uint32 * n)(*stakes)
        self.check(LIB.nw_committee_load(self._ctx, _buf(blob), st, n, slots), "nw_committee_load")
        return list(slots[:n])

    def committee_size(self) -> int:
        return LIB.nw_committee_size(self._ctx)

    def key_window(self) -> int:
        return LIB.nw_key_window(self._ctx)

    def key_negtab(self) -> bool:
        return bool(LIB.nw_key_negtab(self._ctx))

    @staticmethod
    def base_window() -> int:
        return LIB.nw_base_window()

    # -- verification -------------------------------------------------------------------------
    def verify_strict(self, msg: bytes, pk: bytes, sig: bytes) -> bool:
        rc = self.check(LIB.nw_verify_strict(self._ctx, _buf(msg), len(msg), bytes(pk), bytes(sig)),
                        "nw_verify_strict")
        return rc == NW_OK

    def verify_strict_many(self, msgs, pks, sigs):
        n = len(sigs)
        if n == 0:
            return []
        mp = (ctypes.c_char_p * n)(*[bytes(m) for m in msgs])
        ln = (ctypes.c_size_t * n)(*[len(m) for m in msgs])
        ok = (ctypes.c_uint8 * n)()
        self.check(LIB.nw_verify_strict_many(self._ctx, mp, ln, _buf(b"".join(map(bytes, pks))),
                                             _buf(b"".join(map(bytes, sigs))), n, ok), "nw_verify_strict_many")
        return [bool(x) for x in ok]

    def prepare_strict_many_call(self, msgs, pks, sigs):
        """nw_verify_strict_many with the arguments marshalled once (latency measurement: the call
        alone is timed, as a Rust caller passes its slices): returns call() -> ctypes uint8 array."""
        n = len(sigs)
        mp = (ctypes.c_char_p * n)(*[bytes(m) for m in msgs])
        ln = (ctypes.c_size_t * n)(*[len(m) for m in msgs])
        pk_blob, sig_blob = b"".join(map(bytes, pks)), b"".join(map(bytes, sigs))
        ok = (ctypes.c_uint8 * n)()

        def call():
            self.check(LIB.nw_verify_strict_many(self._ctx, mp, ln, pk_blob, sig_blob, n, ok), "nw_verify_strict_many")
            return ok
        return call

    def verify_batch(self, msgs, pks, sigs, zseed: bytes, batch_index: int = 0) -> bool:
        n = len(sigs)
        if len(msgs) != n or len(pks) != n:
            return False   # dalek: ArrayLengthError
        if n == 0:
            return True
        mp = (ctypes.c_char_p * n)(*[bytes(m) for m in msgs])
        ln = (ctypes.c_size_t * n)(*[len(m) for m in msgs])
        rc = self.check(LIB.nw_verify_batch(self._ctx, mp, ln, _buf(b"".join(map(bytes, pks))),
                                            _buf(b"".join(map(bytes, sigs))), n, bytes(zseed), batch_index),
                        "nw_verify_batch")
        return rc == NW_OK

    def verify_certs(self, cert_ranges, sigs_blob: bytes, signer_slots, msgs_blob: bytes, zseed: bytes,
                     cert_base: int = 0):
        """cert_ranges: list of (first_vote, n_votes).  Returns (cert_ok, sig_ok, accepted_stake) lists."""
        nc = len(cert_ranges)
        nsig = len(signer_slots)
        certs = (NwCert * max(nc, 1))(*[NwCert(f, n) for f, n in cert_ranges])
        slots = (ctypes.c_uint32 * max(nsig, 1))(*signer_slots)
        cert_ok = (ctypes.c_uint8 * max(nc, 1))()
        sig_ok = (ctypes.c_uint8 * max(nsig, 1))()
        stake = (ctypes.c_uint64 * max(nc, 1))()
        self.check(LIB.nw_verify_certs(self._ctx, certs, nc, _buf(sigs_blob), slots, _buf(msgs_blob), bytes(zseed),
                                       cert_base, cert_ok, sig_ok, stake), "nw_verify_certs")
        return [bool(x) for x in cert_ok[:nc]], [bool(x) for x in sig_ok[:nsig]], list(stake[:nc])

    def verify_batches(self, batches, msgs, signer_slots, sigs, zseed: bytes, batch_base: int = 0):
        """batches: list of (first, n); msgs: per-signature bytes; signer_slots: key-cache slots;
        sigs: per-signature 64-byte signatures.  Returns (batch_ok list, sig_ok list)."""
        nb, ns = len(batches), len(sigs)
        first = (ctypes.c_uint32 * max(nb, 1))(*[f for f, _ in batches])
        cnt = (ctypes.c_uint32 * max(nb, 1))(*[n for _, n in batches])
        mp = (ctypes.c_char_p * max(ns, 1))(*[bytes(m) for m in msgs])
        ln = (ctypes.c_size_t * max(ns, 1))(*[len(m) for m in msgs])
        slots = (ctypes.c_uint32 * max(ns, 1))(*signer_slots)
        bok = (ctypes.c_uint8 * max(nb, 1))()
        sok = (ctypes.c_uint8 * max(ns, 1))()
        self.check(LIB.nw_verify_batches(self._ctx, nb, first, cnt, mp, ln, slots,
                                         _buf(b"".join(map(bytes, sigs))), bytes(zseed), batch_base, bok, sok),
                   "nw_verify_batches")
        return [bool(x) for x in bok[:nb]], [bool(x) for x in sok[:ns]]

    def verify_batches_np(self, first, counts, msgs, signer_slots, sigs, zseed: bytes, batch_base: int = 0):
        """numpy variant: msgs uint8[N, L] (fixed-length messages, e.g. the worker's 8-byte ones),
        sigs uint8[N, 64], signer_slots uint32[N].  Returns (batch_ok u8[B], sig_ok u8[N])."""
        import numpy as np
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
        slots = np.ascontiguousarray(signer_slots, dtype=np.uint32)
        first = np.ascontiguousarray(first, dtype=np.uint32)
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        n, ml = msgs.shape
        ptrs = (msgs.ctypes.data + np.arange(n, dtype=np.uint64) * ml).astype(np.uint64)
        lens = np.full(n, ml, dtype=np.uint64)
        bok = np.zeros(max(len(first), 1), np.uint8)
        sok = np.zeros(max(n, 1), np.uint8)
        self.check(LIB.nw_verify_batches(self._ctx, len(first), first.ctypes.data, counts.ctypes.data,
                                         ptrs.ctypes.data, lens.ctypes.data, slots.ctypes.data, sigs.ctypes.data,
                                         bytes(zseed), batch_base, bok.ctypes.data, sok.ctypes.data),
                   "nw_verify_batches")
        return bok[:len(first)], sok[:n]

    # -- digests ------------------------------------------------------------------------------
    def sha512(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.check(LIB.nw_sha512(self._ctx, _buf(data), len(data), out), "nw_sha512")
        return out.raw

    def sha512_many(self, messages) -> list:
        n = len(messages)
        if n == 0:
            return []
        offs, lens, pos = [], [], 0
        for m in messages:
            offs.append(pos)
            lens.append(len(m))
            pos += len(m)
        blob = b"".join(bytes(m) for m in messages)
        out = ctypes.create_string_buffer(64 * n)
        self.check(LIB.nw_sha512_many(self._ctx, _buf(blob) if blob else ctypes.c_char_p(b"\0"),
                                      (ctypes.c_uint64 * n)(*offs), (ctypes.c_uint64 * n)(*lens), n, out),
                   "nw_sha512_many")
        return [out.raw[64 * i:64 * (i + 1)] for i in range(n)]

    # -- signing ------------------------------------------------------------------------------
    def sign_many(self, seeds, msgs):
        """RFC 8032 signatures of equal-length (8 or 32 byte) messages; returns (pks, sigs)."""
        n = len(seeds)
        if n == 0:
            return [], []
        mlen = len(msgs[0])
        pk = ctypes.create_string_buffer(32 * n)
        sg = ctypes.create_string_buffer(64 * n)
        self.check(LIB.nw_sign_many(self._ctx, _buf(b"".join(map(bytes, seeds))), _buf(b"".join(map(bytes, msgs))),
                                    mlen, n, pk, sg), "nw_sign_many")
        return ([pk.raw[32 * i:32 * i + 32] for i in range(n)], [sg.raw[64 * i:64 * i + 64] for i in range(n)])


    # -- numpy bulk paths (large synthetic workloads) -------------------------------------------
    def sign_many_np(self, seeds, msgs):
        """seeds: uint8[N,32]; msgs: uint8[N,L] with L in (8, 32).  Returns (pk uint8[N,32], sig uint8[N,64])."""
        import numpy as np
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        n = seeds.shape[0]
        pk = np.empty((n, 32), np.uint8)
        sg = np.empty((n, 64), np.uint8)
        if n:
            self.check(LIB.nw_sign_many(self._ctx, seeds.ctypes.data, msgs.ctypes.data, msgs.shape[1], n,
                                        pk.ctypes.data, sg.ctypes.data), "nw_sign_many")
        return pk, sg

    def committee_load_np(self, pks, stakes=None):
        import numpy as np
        pks = np.ascontiguousarray(pks, dtype=np.uint8)
        n = pks.shape[0]
        slots = np.empty(max(n, 1), np.uint32)
        st = None if stakes is None else np.ascontiguousarray(stakes, dtype=np.uint32)
        self.check(LIB.nw_committee_load(self._ctx, pks.ctypes.data, None if st is None else st.ctypes.data, n,
                                         slots.ctypes.data), "nw_committee_load")
        return slots[:n]

    def verify_certs_np(self, cert_first, cert_n, sigs, signer_slots, msgs, zseed: bytes, cert_base: int = 0):
        """Host-buffer certificate path (numpy in/out): returns (cert_ok u8[C], sig_ok u8[N], stake u64[C])."""
        import numpy as np
        nc = len(cert_first)
        certs = np.empty((nc, 2), np.uint32)
        certs[:, 0] = cert_first
        certs[:, 1] = cert_n
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
        slots = np.ascontiguousarray(signer_slots, dtype=np.uint32)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        cert_ok = np.zeros(max(nc, 1), np.uint8)
        sig_ok = np.zeros(max(len(slots), 1), np.uint8)
        stake = np.zeros(max(nc, 1), np.uint64)
        self.check(LIB.nw_verify_certs(self._ctx, certs.ctypes.data, nc, sigs.ctypes.data, slots.ctypes.data,
                                       msgs.ctypes.data, bytes(zseed), cert_base, cert_ok.ctypes.data,
                                       sig_ok.ctypes.data, stake.ctypes.data), "nw_verify_certs")
        return cert_ok[:nc], sig_ok[:len(slots)], stake[:nc]

    def verify_certs_dev(self, ncerts, d_first, d_n, nsigs, d_sig, d_signer, d_msg, zseed: bytes, cert_base,
                         d_cert_ok, d_flags, d_stake, stream, d_status=None):
        """Device-pointer path (ints = device addresses, e.g. torch ``data_ptr()``).  With
        ``d_status`` None the device-side input check is synchronous and a bad input raises
        DeviceError (NW_ERR_ARG); with a device uint32 address it is written in stream order and the
        call only enqueues."""
        self.check(LIB.nw_verify_certs_dev(self._ctx, ncerts, d_first, d_n, nsigs, d_sig, d_signer, d_msg,
                                           bytes(zseed), cert_base, d_cert_ok, d_flags, d_stake, d_status, stream),
                   "nw_verify_certs_dev")

    def verify_batches_pk(self, counts, msgs, pks, sigs, zseed: bytes, batch_base: int = 0):
        """Batches over arbitrary keys (variable-base Pippenger path): batch b is the next
        counts[b] signatures.  msgs: list of bytes; pks/sigs: lists (or one joined bytes blob).
        Returns a list of bools."""
        nb = len(counts)
        n = sum(counts)
        if nb == 0:
            return []
        mp = (ctypes.c_char_p * max(n, 1))(*[bytes(m) for m in msgs])
        ln = (ctypes.c_size_t * max(n, 1))(*[len(m) for m in msgs])
        cnt = (ctypes.c_uint32 * nb)(*counts)
        pkb = pks if isinstance(pks, (bytes, bytearray)) else b"".join(map(bytes, pks))
        sgb = sigs if isinstance(sigs, (bytes, bytearray)) else b"".join(map(bytes, sigs))
        ok = (ctypes.c_uint8 * nb)()
        self.check(LIB.nw_verify_batches_pk(self._ctx, nb, cnt, mp, ln, _buf(bytes(pkb)), _buf(bytes(sgb)),
                                            bytes(zseed), batch_base, ok), "nw_verify_batches_pk")
        return [bool(x) for x in ok]

    def verify_batches_pk_np(self, counts, msgs, pks, sigs, zseed: bytes, batch_base: int = 0):
        """numpy variant: msgs uint8[N, L] (fixed length), pks uint8[N, 32], sigs uint8[N, 64]."""
        import numpy as np
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        pks = np.ascontiguousarray(pks, dtype=np.uint8)
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        n, ml = msgs.shape
        ptrs = (msgs.ctypes.data + np.arange(n, dtype=np.uint64) * ml).astype(np.uint64)
        lens = np.full(n, ml, dtype=np.uint64)
        ok = np.zeros(max(len(counts), 1), np.uint8)
        self.check(LIB.nw_verify_batches_pk(self._ctx, len(counts), counts.ctypes.data, ptrs.ctypes.data,
                                            lens.ctypes.data, pks.ctypes.data, sigs.ctypes.data, bytes(zseed),
                                            batch_base, ok.ctypes.data), "nw_verify_batches_pk")
        return ok[:len(counts)]

    def verify_batch_partial(self, msgs, pks, sigs, zseed: bytes, batch_index: int, z_offset: int):
        """One shard's share of a split batch: returns (point bytes[160], bad)."""
        n = len(sigs)
        mp = (ctypes.c_char_p * max(n, 1))(*[bytes(m) for m in msgs])
        ln = (ctypes.c_size_t * max(n, 1))(*[len(m) for m in msgs])
        pt = ctypes.create_string_buffer(POINT_BYTES)
        bad = ctypes.c_int(0)
        self.check(LIB.nw_verify_batch_partial(self._ctx, mp, ln, _buf(b"".join(map(bytes, pks))),
                                               _buf(b"".join(map(bytes, sigs))), n, bytes(zseed), batch_index,
                                               z_offset, pt, ctypes.byref(bad)), "nw_verify_batch_partial")
        return pt.raw, bool(bad.value)

    def prepare_batch_call(self, msgs, pks, sigs):
        """Marshal one nw_verify_batch call once; returns ``call(zseed, batch_index) -> bool`` that
        only crosses the ABI (latency legs: the cost a Rust caller pays, not Python's packing)."""
        import numpy as np
        n = len(sigs)
        keep = [np.ascontiguousarray(np.frombuffer(b"".join(bytes(m) for m in msgs), np.uint8)),
                np.ascontiguousarray(np.frombuffer(b"".join(bytes(k) for k in pks), np.uint8)),
                np.ascontiguousarray(np.frombuffer(b"".join(bytes(s) for s in sigs), np.uint8))]
        lens = np.array([len(m) for m in msgs], np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        ptrs = (keep[0].ctypes.data + offs).astype(np.uint64)
        keep += [lens, ptrs]
        lib, ctx = LIB, self._ctx

        def call(zseed: bytes, batch_index: int = 0) -> bool:
            _ = keep
            return self.check(lib.nw_verify_batch(ctx, ptrs.ctypes.data, lens.ctypes.data, keep[1].ctypes.data,
                                                  keep[2].ctypes.data, n, zseed, batch_index),
                              "nw_verify_batch") == NW_OK
        return call

    def prepare_batches_pk_call(self, counts, msgs, pks, sigs):
        """Marshal one nw_verify_batches_pk call once (fixed-length numpy messages); returns
        ``call(zseed, batch_base) -> uint8[nb]`` that only crosses the ABI."""
        import numpy as np
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        pks = np.ascontiguousarray(pks, dtype=np.uint8)
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        n, ml = msgs.shape
        ptrs = (msgs.ctypes.data + np.arange(n, dtype=np.uint64) * ml).astype(np.uint64)
        lens = np.full(n, ml, dtype=np.uint64)
        ok = np.zeros(max(len(counts), 1), np.uint8)
        keep = (msgs, pks, sigs, counts, ptrs, lens)
        lib, ctx, nb = LIB, self._ctx, len(counts)
        args = (counts.ctypes.data, ptrs.ctypes.data, lens.ctypes.data, pks.ctypes.data, sigs.ctypes.data)

        def call(zseed: bytes, batch_base: int = 0):
            _ = keep
            self.check(lib.nw_verify_batches_pk(ctx, nb, *args, zseed, batch_base, ok.ctypes.data),
                       "nw_verify_batches_pk")
            return ok[:nb]
        return call

    def points_sum_is_identity(self, points) -> bool:
        blob = b"".join(bytes(p) for p in points)
        r = ctypes.c_int(0)
        self.check(LIB.nw_points_sum_is_identity(self._ctx, _buf(blob), len(points), ctypes.byref(r)),
                   "nw_points_sum_is_identity")
        return bool(r.value)

    def profile_enable(self, on: bool = True):
        self.check(LIB.nw_profile_enable(self._ctx, 1 if on else 0), "nw_profile_enable")

    def profile_read(self):
        """(summed k_verify device ms, launches, signatures in those launches) since the last read;
        synchronizes the events."""
        ms = ctypes.c_double(0)
        n = ctypes.c_uint64(0)
        sigs = ctypes.c_uint64(0)
        if not hasattr(LIB, "nw_profile_read_sigs"):
            self.check(LIB.nw_profile_read(self._ctx, ctypes.byref(ms), ctypes.byref(n)), "nw_profile_read")
            return ms.value, n.value, None
        self.check(LIB.nw_profile_read_sigs(self._ctx, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(sigs)),
                   "nw_profile_read_sigs")
        return ms.value, n.value, sigs.value

    def sha512_many_submit(self, messages) -> "DigestJob":
        """nw_sha512_many_async: enqueue the digests of ``messages`` (bytes-like objects or uint8
        numpy arrays, kept referenced until the job is waited for) and return at once."""
        return DigestJob(self, messages)

    def sha512_many_dev(self, d_base, d_off, d_len, n, d_out, stream):
        self.check(LIB.nw_sha512_many_dev(self._ctx, d_base, d_off, d_len, n, d_out, stream), "nw_sha512_many_dev")

    # -- primary certificate path (nw_cert_batch_verify) ----------------------------------------
    def cert_batch_verify(self, batch: "CertBatch", zseed: bytes, cert_base: int = 0):
        """NW_DAG_* verdict per certificate of a decoded batch (GPU: digests, header signatures,
        vote batches)."""
        n = len(batch)
        out = (ctypes.c_int32 * max(n, 1))()
        self.check(LIB.nw_cert_batch_verify(self._ctx, batch.handle, _buf(bytes(zseed)), cert_base, out),
                   "nw_cert_batch_verify")
        return list(out[:n])


class DigestJob:
    """One nw_sha512_many_async submission in flight.  ``done()`` polls; ``wait()`` returns the
    64-byte digests in submission order (exactly once).  The message buffers stay referenced by
    the job until then, as the ABI requires."""

    def __init__(self, engine: Engine, messages):
        import numpy as np
        self._engine = engine
        self._msgs = [self._as_bytes(m) for m in messages]
        n = len(self._msgs)
        self.n = n
        self._ptrs = np.array([m.ctypes.data if m.size else 0 for m in self._msgs], np.uint64)
        self._lens = np.array([m.size for m in self._msgs], np.uint64)
        self._out = np.zeros((max(n, 1), 64), np.uint8)
        self._job = ctypes.c_void_p()
        engine.check(LIB.nw_sha512_many_async(engine.handle, self._ptrs.ctypes.data, self._lens.ctypes.data, n,
                                              self._out.ctypes.data, ctypes.byref(self._job)), "nw_sha512_many_async")

    @staticmethod
    def _as_bytes(m):
        """A flat uint8 view of one message: the pointer and byte length the ABI gets must describe
        its bytes.  Non-uint8 or non-contiguous arrays raise rather than hash the wrong bytes."""
        import numpy as np
        if isinstance(m, np.ndarray):
            if m.dtype != np.uint8 or not m.flags.c_contiguous:
                raise TypeError("DigestJob: messages must be bytes-like or C-contiguous uint8 arrays")
            return m.reshape(-1)
        return np.frombuffer(m, np.uint8)

    def done(self) -> bool:
        if not self._job:
            return True
        rc = LIB.nw_job_done(self._job)
        if rc < 0 or rc > 1:
            raise DeviceError("nw_job_done failed (rc=%d)" % rc)
        return rc == 1

    def wait(self) -> list:
        if self._job:
            job, self._job = self._job, ctypes.c_void_p()
            self._engine.check(LIB.nw_job_wait(job), "nw_job_wait")
            self._msgs = None
        return [bytes(self._out[i]) for i in range(self.n)]

    def __del__(self):
        try:
            if self._job:
                LIB.nw_job_wait(self._job)   # a job must be waited for exactly once
        except Exception:
            pass


class CommitteeABI:
    """nw_committee view of (names, stakes, worker id lists); keeps the buffers alive."""

    def __init__(self, names, stakes, workers):
        names = [bytes(k) for k in names]
        n = len(names)
        self._names = b"".join(names)
        self._stake = (ctypes.c_uint32 * max(n, 1))(*stakes)
        first, ids = [0], []
        for ws in workers:
            ids.extend(sorted(ws))
            first.append(len(ids))
        self._first = (ctypes.c_uint32 * len(first))(*first)
        self._ids = (ctypes.c_uint32 * max(len(ids), 1))(*ids)
        self.struct = NwCommittee(n, ctypes.cast(ctypes.c_char_p(self._names), ctypes.c_void_p) if n else None,
                                  ctypes.cast(self._stake, ctypes.c_void_p), ctypes.cast(self._first, ctypes.c_void_p),
                                  ctypes.cast(self._ids, ctypes.c_void_p))


class CertBatch:
    """Host-side decode of bincode PrimaryMessage frames (nw_cert_batch_decode: C++, no GPU)."""

    def __init__(self, committee: CommitteeABI, frames):
        frames = [bytes(f) for f in frames]
        n = len(frames)
        self._frames = frames
        ptrs = (ctypes.c_char_p * max(n, 1))(*frames)
        lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in frames])
        self._h = ctypes.c_void_p()
        rc = LIB.nw_cert_batch_decode(ctypes.byref(committee.struct), ptrs, lens, n, ctypes.byref(self._h))
        if rc != NW_OK:
            raise DeviceError("nw_cert_batch_decode failed (rc=%d)" % rc)

    @property
    def handle(self):
        return self._h

    def __len__(self):
        return LIB.nw_cert_batch_size(self._h)

    def view(self, i: int) -> dict:
        v = NwCertView()
        if LIB.nw_cert_batch_view(self._h, i, ctypes.byref(v)) != NW_OK:
            raise IndexError(i)

        def rd(p, k):
            return ctypes.string_at(p, k) if k else b""
        return {"status": v.status, "header_error": v.header_error, "quorum_error": v.quorum_error,
                "round": v.round, "author": rd(v.author, 32), "header_id": rd(v.header_id, 32),
                "header_sig": rd(v.header_sig, 64), "header_preimage": rd(v.header_preimage, v.header_preimage_len),
                "cert_preimage": rd(v.cert_preimage, 72),
                "votes": [(rd(v.vote_keys + 32 * j, 32), rd(v.vote_sigs + 64 * j, 64)) for j in range(v.n_votes)]}

    def close(self):
        if self._h:
            LIB.nw_cert_batch_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default: Optional[Engine] = None
_default_lock = threading.Lock()


def default_engine() -> Engine:
    """Process-wide engine on this process's GPU (LOCAL_RANK, else the current device)."""
    global _default
    with _default_lock:
        if _default is None:
            dev = int(os.environ.get("LOCAL_RANK", "-1"))
            _default = Engine(device=dev)
        return _default


def version() -> str:
    return LIB.nw_version().decode()
