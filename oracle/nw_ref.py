"""ctypes wrapper of oracle/libnwref.so — the C restatement of dalek 1.0.1 (TEST / BASELINE
INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg, never by the product)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "libnwref.so")
if not os.path.exists(_PATH):
    raise ImportError("oracle/libnwref.so not built (make -C oracle)")
_lib = ctypes.CDLL(_PATH)
_P, _S = ctypes.c_void_p, ctypes.c_size_t
_lib.nwr_verify_strict.argtypes = [_P, _S, _P, _P]
_lib.nwr_crypto_verify_batch.argtypes = [_P, _S, _P, _P, _S, _P, ctypes.c_uint64]
_lib.nwr_decompress.argtypes = [_P, _P]
_lib.nwr_sha512.argtypes = [_P, _S, _P]
_lib.nwr_verify_batch_msgs.argtypes = [_P, _P, _P, _P, _S, _P, ctypes.c_uint64]
_lib.nwr_verify_certs.argtypes = [_P, _P, _P, _P, _P, _P, _P, _S, _P, ctypes.c_uint64, ctypes.c_int, _P]
_lib.nwr_init()


def verify_strict(pk: bytes, msg: bytes, sig: bytes) -> bool:
    return bool(_lib.nwr_verify_strict(msg, len(msg), pk, sig))


def crypto_verify_batch(digest: bytes, votes, zseed: bytes, batch_index: int = 0) -> bool:
    n = len(votes)
    pks = b"".join(k for k, _ in votes)
    sigs = b"".join(s for _, s in votes)
    return bool(_lib.nwr_crypto_verify_batch(digest, len(digest), pks or None, sigs or None, n, zseed, batch_index))


def prepare_crypto_verify_batch(digest: bytes, pks, sigs):
    """crypto_verify_batch with the vote arrays joined once (the latency comparator times the call
    alone): returns call(zseed, batch_index) -> bool."""
    n = len(sigs)
    pk_blob, sig_blob = b"".join(bytes(k) for k in pks), b"".join(bytes(s) for s in sigs)
    pk_buf = ctypes.create_string_buffer(pk_blob, max(1, len(pk_blob)))
    sig_buf = ctypes.create_string_buffer(sig_blob, max(1, len(sig_blob)))

    def call(zseed: bytes, batch_index: int = 0) -> bool:
        return bool(_lib.nwr_crypto_verify_batch(digest, len(digest), pk_buf, sig_buf, n, zseed, batch_index))
    return call


def verify_batch_msgs(msgs, pks, sigs, zseed: bytes, batch_index: int = 0) -> bool:
    """dalek::verify_batch with per-signature messages (worker/src/processor.rs:78)."""
    n = len(sigs)
    mp = (ctypes.c_char_p * max(n, 1))(*[bytes(m) for m in msgs])
    ln = (ctypes.c_size_t * max(n, 1))(*[len(m) for m in msgs])
    return bool(_lib.nwr_verify_batch_msgs(mp, ln, b"".join(pks) or None, b"".join(sigs) or None, n, zseed,
                                           batch_index))


def decompress(b: bytes):
    out = ctypes.create_string_buffer(32)
    return out.raw if _lib.nwr_decompress(b, out) else None


def sha512(m: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    _lib.nwr_sha512(m, len(m), out)
    return out.raw


def verify_certs(cs, com, sel, zseed: bytes, threads: int, cert_base: int = 0):
    """Batch-verify the selected certificates of a narwhal_amd.workload.Certificates on
    ``threads`` host threads (per-vote key decompression, dalek's batch equation)."""
    sel = np.ascontiguousarray(np.asarray(sel, dtype=np.uint32))
    out = np.zeros(len(sel), np.uint8)
    msgs = np.ascontiguousarray(cs.msgs)
    first = np.ascontiguousarray(cs.cert_first, dtype=np.uint32)
    nv = np.ascontiguousarray(cs.cert_n, dtype=np.uint32)
    pks = np.ascontiguousarray(com.pks)
    signer = np.ascontiguousarray(cs.signer, dtype=np.uint32)
    sigs = np.ascontiguousarray(cs.sigs)
    _lib.nwr_verify_certs(msgs.ctypes.data, first.ctypes.data, nv.ctypes.data, pks.ctypes.data, signer.ctypes.data,
                          sigs.ctypes.data, sel.ctypes.data, len(sel), zseed, cert_base, threads, out.ctypes.data)
    return out.astype(bool).tolist()
