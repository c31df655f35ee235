"""Host mirror of the reference ``crypto`` crate (crypto/src/lib.rs) over libnwcrypto.

Same names, argument meaning and error behaviour as the Rust API, so callers (and the parity
tests, which read like crypto/src/tests/crypto_tests.rs) switch by import:

=========================================  ==============================================
reference (crypto/src/lib.rs)              here
=========================================  ==============================================
``CryptoError`` (:18)                      ``CryptoError`` exception
``Digest`` (:22-56)                        ``Digest``
``Hash`` trait (:59-62)                    ``Hash`` protocol (``digest()``)
``PublicKey`` (:66-118)                    ``PublicKey`` (base64 import/export)
``SecretKey`` (:121-160)                   ``SecretKey``
``generate_production_keypair`` (:162)     ``generate_production_keypair``
``generate_keypair`` (:166-175)            ``generate_keypair``
``Signature::new`` (:185-191)              ``Signature.new`` (GPU signing kernel)
``Signature::verify`` (:200-204)           ``Signature.verify`` -> strict verify on the GPU
``Signature::verify_batch`` (:206-219)     ``Signature.verify_batch`` -> batch verify on the GPU
``SignatureService`` (:222-250)            ``SignatureService``
=========================================  ==============================================

``verify``/``verify_batch`` return None on success and raise ``CryptoError`` on failure
(the Rust ``Result<(), CryptoError>``).  The batch coefficients are drawn from a fresh OS random
seed per call (the reference uses ``thread_rng``); pass ``zseed=`` to pin them for parity tests.
"""
from __future__ import annotations

import asyncio
import base64
import os
from typing import Iterable, Optional, Tuple

from . import _lib


class CryptoError(Exception):
    """``ed25519::Error`` — opaque signature error (crypto/src/lib.rs:18)."""


class Digest:
    """32-byte hash digest (crypto/src/lib.rs:22)."""

    __slots__ = ("_b",)

    def __init__(self, b: bytes = bytes(32)):
        b = bytes(b)
        if len(b) != 32:
            raise ValueError("Digest must be 32 bytes")
        self._b = b

    @classmethod
    def try_from(cls, item: bytes) -> "Digest":
        return cls(item)

    def to_vec(self) -> bytes:
        return self._b

    def size(self) -> int:
        return 32

    def __bytes__(self):
        return self._b

    def __eq__(self, other):
        return isinstance(other, Digest) and self._b == other._b

    def __lt__(self, other):
        return self._b < other._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):   # fmt::Debug
        return base64.b64encode(self._b).decode()

    def __str__(self):    # fmt::Display
        return base64.b64encode(self._b).decode()[:16]


class Hash:
    """The ``Hash`` trait: implementors provide ``digest() -> Digest``."""

    def digest(self) -> Digest:  # pragma: no cover - interface
        raise NotImplementedError


class PublicKey:
    """Ed25519 public key bytes (crypto/src/lib.rs:66)."""

    __slots__ = ("_b",)

    def __init__(self, b: bytes = bytes(32)):
        b = bytes(b)
        if len(b) != 32:
            raise ValueError("PublicKey must be 32 bytes")
        self._b = b

    def encode_base64(self) -> str:
        return base64.b64encode(self._b).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "PublicKey":
        raw = base64.b64decode(s)
        if len(raw) < 32:
            raise ValueError("InvalidLength")
        return cls(raw[:32])

    def __bytes__(self):
        return self._b

    def __eq__(self, other):
        return isinstance(other, PublicKey) and self._b == other._b

    def __lt__(self, other):
        return self._b < other._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):
        return self.encode_base64()

    def __str__(self):
        return self.encode_base64()[:16]


class SecretKey:
    """64-byte secret key = seed || public key, dalek ``Keypair::to_bytes`` (crypto/src/lib.rs:121)."""

    __slots__ = ("_b",)

    def __init__(self, b: bytes):
        b = bytes(b)
        if len(b) != 64:
            raise ValueError("SecretKey must be 64 bytes")
        self._b = b

    def encode_base64(self) -> str:
        return base64.b64encode(self._b).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "SecretKey":
        raw = base64.b64decode(s)
        if len(raw) < 64:
            raise ValueError("InvalidLength")
        return cls(raw[:64])

    @property
    def seed(self) -> bytes:
        return self._b[:32]

    def __eq__(self, other):
        return isinstance(other, SecretKey) and self._b == other._b

    def __bytes__(self):
        return self._b


def _engine():
    return _lib.default_engine()


def generate_keypair(csprng) -> Tuple[PublicKey, SecretKey]:
    """dalek ``Keypair::generate``: 32 bytes from ``csprng`` (a callable ``n -> bytes``, e.g. a
    ChaCha20 ``fill_bytes``) become the secret seed; the public key is derived on the GPU."""
    seed = bytes(csprng(32))
    pks, _ = _engine().sign_many([seed], [bytes(32)])
    return PublicKey(pks[0]), SecretKey(seed + pks[0])


def generate_production_keypair() -> Tuple[PublicKey, SecretKey]:
    return generate_keypair(os.urandom)


class Signature:
    """Ed25519 signature ``{part1: R, part2: S}`` (crypto/src/lib.rs:178-182); default = zeros."""

    __slots__ = ("part1", "part2")

    def __init__(self, part1: bytes = bytes(32), part2: bytes = bytes(32)):
        self.part1 = bytes(part1)
        self.part2 = bytes(part2)

    @classmethod
    def default(cls) -> "Signature":
        return cls()

    @classmethod
    def from_bytes(cls, b: bytes) -> "Signature":
        return cls(b[:32], b[32:64])

    @classmethod
    def new(cls, digest: Digest, secret: SecretKey) -> "Signature":
        """``Signature::new``: RFC 8032 signature of the 32-byte digest."""
        _, sigs = _engine().sign_many([secret.seed], [bytes(digest)])
        return cls.from_bytes(sigs[0])

    def flatten(self) -> bytes:
        return self.part1 + self.part2

    def __eq__(self, other):
        return isinstance(other, Signature) and self.flatten() == other.flatten()

    def __repr__(self):
        return "Signature { part1: %s, part2: %s }" % (self.part1.hex(), self.part2.hex())

    def verify(self, digest: Digest, public_key: PublicKey) -> None:
        """``Signature::verify`` -> ed25519 parse, PublicKey::from_bytes, verify_strict."""
        if not _engine().verify_strict(bytes(digest), bytes(public_key), self.flatten()):
            raise CryptoError("signature verification failed")

    @staticmethod
    def verify_batch(digest: Digest, votes: Iterable[Tuple[PublicKey, "Signature"]],
                     zseed: Optional[bytes] = None, batch_index: int = 0) -> None:
        """``Signature::verify_batch``: all votes sign ``digest``; one verdict, no culprit."""
        votes = list(votes)
        if not votes:
            return None
        d = bytes(digest)
        ok = _engine().verify_batch([d] * len(votes), [bytes(k) for k, _ in votes], [s.flatten() for _, s in votes],
                                    zseed if zseed is not None else os.urandom(32), batch_index)
        if not ok:
            raise CryptoError("batch verification failed")
        return None


class SignatureService:
    """Holds the node's secret key and signs digests on request (crypto/src/lib.rs:222-250)."""

    def __init__(self, secret: SecretKey):
        self._secret = secret

    async def request_signature(self, digest: Digest) -> Signature:
        loop = asyncio.get_running_loop()
        return await loop.run_in_executor(None, Signature.new, digest, self._secret)

    def request_signature_sync(self, digest: Digest) -> Signature:
        return Signature.new(digest, self._secret)


def sha512(data: bytes) -> bytes:
    """``ed25519_dalek::Sha512::digest`` on the GPU (callers truncate to 32 bytes)."""
    return _engine().sha512(bytes(data))


def digest_of(data: bytes) -> Digest:
    """``Digest(Sha512::digest(data)[..32])`` — e.g. crypto_tests.rs:8-12, processor.rs:65."""
    return Digest(sha512(data)[:32])
