"""Synthetic committees and certificates, generated on the GPU.

* Validator secret seeds follow the reference fixture convention — the ChaCha20 keystream of
  ``StdRng::from_seed([0; 32])`` (crypto/src/tests/crypto_tests.rs:26-29) — extended past 4 keys,
  so validators 0..3 are exactly the reference's ``keys()``.
* Certificate j: origin = j mod N, round = j, ``header.id = SHA512("hdr" || u64le(j))[..32]``,
  message = ``SHA512(id || u64le(round) || origin)[..32]`` (the vote/certificate digest of
  primary/src/messages.rs:145-153,226-234); votes come from validators origin, origin+1, ...
* Digests and signatures are computed by libnwcrypto (GPU SHA-512 and signing kernels).
"""
from __future__ import annotations

import dataclasses
import struct

import numpy as np

from . import _lib


def _chacha20_keystream(nbytes: int) -> bytes:
    """ChaCha20 (RFC 8439 block function, key = 0^32, nonce = 0) keystream, vectorized over blocks."""
    nblk = (nbytes + 63) // 64
    const = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], np.uint32)
    st = np.zeros((nblk, 16), np.uint32)
    st[:, 0:4] = const
    st[:, 12] = np.arange(nblk, dtype=np.uint32)
    x = st.copy()

    def rotl(v, n):
        return (v << np.uint32(n)) | (v >> np.uint32(32 - n))

    def qr(a, b, c, d):
        x[:, a] += x[:, b]; x[:, d] = rotl(x[:, d] ^ x[:, a], 16)
        x[:, c] += x[:, d]; x[:, b] = rotl(x[:, b] ^ x[:, c], 12)
        x[:, a] += x[:, b]; x[:, d] = rotl(x[:, d] ^ x[:, a], 8)
        x[:, c] += x[:, d]; x[:, b] = rotl(x[:, b] ^ x[:, c], 7)

    with np.errstate(over="ignore"):
        for _ in range(10):
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
        out = (x + st).astype("<u4")
    return out.tobytes()[:nbytes]


@dataclasses.dataclass
class Committee:
    seeds: np.ndarray    # uint8[N, 32]
    pks: np.ndarray      # uint8[N, 32]
    stake: np.ndarray    # uint32[N]

    @property
    def size(self) -> int:
        return self.pks.shape[0]

    def quorum_threshold(self) -> int:
        """config/src/lib.rs:189-194: 2 * total / 3 + 1."""
        return int(2 * int(self.stake.sum()) // 3 + 1)


@dataclasses.dataclass
class Certificates:
    cert_first: np.ndarray   # uint32[C]
    cert_n: np.ndarray       # uint32[C]
    msgs: np.ndarray         # uint8[C, 32]  certificate digest signed by every vote
    signer: np.ndarray       # uint32[S]     committee index of each vote
    sigs: np.ndarray         # uint8[S, 64]

    @property
    def ncerts(self) -> int:
        return self.cert_first.shape[0]

    @property
    def nsigs(self) -> int:
        return self.signer.shape[0]


def make_committee(n: int, engine: "_lib.Engine" = None, stake: int = 1) -> Committee:
    eng = engine or _lib.default_engine()
    seeds = np.frombuffer(_chacha20_keystream(32 * n), np.uint8).reshape(n, 32).copy()
    pks, _ = eng.sign_many_np(seeds, np.zeros((n, 32), np.uint8))
    return Committee(seeds=seeds, pks=pks, stake=np.full(n, stake, np.uint32))


def certificate_digests(ncerts: int, committee: Committee, engine: "_lib.Engine" = None,
                        first_cert: int = 0) -> np.ndarray:
    """message of certificate j (global index first_cert + j), computed with GPU SHA-512."""
    eng = engine or _lib.default_engine()
    n = committee.size
    idx = range(first_cert, first_cert + ncerts)
    ids = eng.sha512_many([b"hdr" + struct.pack("<Q", j) for j in idx])
    pre = [ids[k][:32] + struct.pack("<Q", j) + bytes(committee.pks[j % n]) for k, j in enumerate(idx)]
    d = eng.sha512_many(pre)
    return np.frombuffer(b"".join(x[:32] for x in d), np.uint8).reshape(ncerts, 32).copy()


def make_certificates(committee: Committee, ncerts: int, votes_per_cert: int, engine: "_lib.Engine" = None,
                      first_cert: int = 0, chunk: int = 1 << 20) -> Certificates:
    eng = engine or _lib.default_engine()
    n = committee.size
    if votes_per_cert > n:
        raise ValueError("votes_per_cert > committee size")
    msgs = certificate_digests(ncerts, committee, eng, first_cert)
    cert_n = np.full(ncerts, votes_per_cert, np.uint32)
    cert_first = (np.arange(ncerts, dtype=np.uint64) * votes_per_cert).astype(np.uint32)
    origin = (np.arange(first_cert, first_cert + ncerts, dtype=np.int64) % n)
    signer = ((origin[:, None] + np.arange(votes_per_cert)[None, :]) % n).astype(np.uint32).reshape(-1)
    cert_of = np.repeat(np.arange(ncerts), votes_per_cert)
    total = signer.shape[0]
    sigs = np.empty((total, 64), np.uint8)
    for s in range(0, total, chunk):
        e = min(total, s + chunk)
        _, sg = eng.sign_many_np(committee.seeds[signer[s:e]], msgs[cert_of[s:e]])
        sigs[s:e] = sg
    return Certificates(cert_first=cert_first, cert_n=cert_n, msgs=msgs, signer=signer, sigs=sigs)


def worker_batch(n_tx: int, tx_size: int, batch_id: int = 0) -> bytes:
    """bincode ``WorkerMessage::Batch`` of benchmark-client transactions
    (node/src/benchmark_client.rs:166-186: 0xFFFFFFFF then a BE counter, zero-padded;
    worker/src/batch_maker.rs:118-119 serialization)."""
    parts = [struct.pack("<IQ", 0, n_tx)]
    for t in range(n_tx):
        tx = struct.pack(">II", 0xFFFFFFFF, (batch_id * n_tx + t) & 0xFFFFFFFF).ljust(tx_size, b"\0")
        parts.append(struct.pack("<Q", tx_size))
        parts.append(tx)
    return b"".join(parts)


def worker_batches_np(n_batches: int, n_tx: int = 977, tx_size: int = 512) -> "np.ndarray":
    """``n_batches`` serialized worker batches as one uint8[n_batches, 12 + n_tx * (8 + tx_size)]
    array, byte-identical to ``worker_batch(n_tx, tx_size, b)`` for b = 0 .. n_batches - 1
    (vectorized: the C4 node load is 10,000 x 508,052 B)."""
    rec = 8 + tx_size
    blen = 12 + n_tx * rec
    out = np.zeros((n_batches, blen), np.uint8)
    out[:, 4:12] = np.frombuffer(struct.pack("<Q", n_tx), np.uint8)
    body = out[:, 12:].reshape(n_batches, n_tx, rec)
    body[:, :, 0:8] = np.frombuffer(struct.pack("<Q", tx_size), np.uint8)
    body[:, :, 8:12] = 0xFF
    ctr = (np.arange(n_batches, dtype=np.uint64)[:, None] * n_tx + np.arange(n_tx, dtype=np.uint64)[None, :])
    ctr = (ctr & 0xFFFFFFFF).astype(">u4")
    body[:, :, 12:16] = ctr.view(np.uint8).reshape(n_batches, n_tx, 4)
    return out
