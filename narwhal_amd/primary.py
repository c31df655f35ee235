"""Host mirror of the reference's certificate / header / vote callers of the hot path.

Follows primary/src/messages.rs (Header :13-84, Vote :105-153, Certificate :168-256),
primary/src/error.rs (DagError) and config/src/lib.rs (Committee :161-229), with the reference's
bincode wire format (PrimaryMessage, primary/src/primary.rs:33-38).  Every digest and signature
check runs on the GPU through libnwcrypto:

* ``Header.verify`` / ``Vote.verify`` / ``Certificate.verify`` are the one-message forms, with the
  reference's check order and error kinds;
* ``verify_certificates`` is the Core-side batching of SURVEY §8(f) item 3: the same checks for many
  certificates with ONE GPU SHA-512 submission (header + certificate digests, §8(f) item 2), ONE
  strict-verify submission (header signatures) and ONE certificate batch-verify submission.

This module holds only host logic (ordering, stake sums, wire format); it never computes a digest
or a verdict on the CPU.
"""
from __future__ import annotations

import base64
import struct
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib


# ----------------------------------------------------------------------------- errors (error.rs)
class DagError(Exception):
    """primary/src/error.rs:25-60."""


class InvalidSignature(DagError):
    pass


class InvalidHeaderId(DagError):
    pass


class MalformedHeader(DagError):
    pass


class UnknownAuthority(DagError):
    pass


class AuthorityReuse(DagError):
    pass


class CertificateRequiresQuorum(DagError):
    pass


class SerializationError(DagError):
    pass


# ----------------------------------------------------------------------------- committee (config)
class Committee:
    """config/src/lib.rs:161-229: authorities keyed by public key (BTreeMap: byte order)."""

    def __init__(self, authorities: Dict[bytes, Tuple[int, Iterable[int]]]):
        self.authorities = {bytes(k): (int(st), frozenset(ws)) for k, (st, ws) in sorted(authorities.items())}

    def size(self) -> int:
        return len(self.authorities)

    def stake(self, name: bytes) -> int:
        a = self.authorities.get(bytes(name))
        return a[0] if a else 0

    def quorum_threshold(self) -> int:
        total = sum(st for st, _ in self.authorities.values())
        return 2 * total // 3 + 1

    def validity_threshold(self) -> int:
        total = sum(st for st, _ in self.authorities.values())
        return (total + 2) // 3

    def has_worker(self, name: bytes, worker_id: int) -> bool:
        a = self.authorities.get(bytes(name))
        return a is not None and worker_id in a[1]

    def keys(self) -> List[bytes]:
        return list(self.authorities.keys())


# ----------------------------------------------------------------------------- wire format (bincode)
class _Reader:
    def __init__(self, buf: bytes):
        self.b = memoryview(buf)
        self.p = 0

    def take(self, n: int) -> bytes:
        if self.p + n > len(self.b):
            raise SerializationError("truncated message")
        out = bytes(self.b[self.p:self.p + n])
        self.p += n
        return out

    def u32(self) -> int:
        return struct.unpack("<I", self.take(4))[0]

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]

    def public_key(self) -> bytes:
        """PublicKey serializes as its base64 string (crypto/src/lib.rs:94-112)."""
        raw = _b64_decode(self.take(self.u64()))
        if raw is None:
            raise SerializationError("bad base64 public key")
        if len(raw) < 32:
            raise SerializationError("public key too short")
        return raw[:32]


_B64 = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"


def _b64_decode(s: bytes) -> Optional[bytes]:
    """base64 0.13 STANDARD decode (crypto/src/lib.rs:73) as restated in nw_primary.cpp b64_decode:
    '=' only in the final quantum at quad positions 2 and 3 with nothing but '=' after it, padding
    optional and not required to complete the quad; a 1-symbol final quantum and non-zero trailing
    bits are rejected.  None = decode error."""
    s = bytes(s)
    n = len(s)
    m = s.find(b"=")
    m = n if m < 0 else m
    if any(s[i:i + 1] != b"=" or i % 4 < 2 for i in range(m, n)) or n - m > 2 or m % 4 == 1:
        return None
    if any(c not in _B64 for c in s[:m]):
        return None
    full = s[:m] + b"=" * (-m % 4)
    out = base64.b64decode(full)
    # trailing bits of the last symbol must be zero (re-encoding reproduces the symbols)
    if base64.b64encode(out)[:m] != s[:m]:
        return None
    return out


def _pk_bytes(pk: bytes) -> bytes:
    s = base64.b64encode(bytes(pk))
    return struct.pack("<Q", len(s)) + s


# ----------------------------------------------------------------------------- messages
class Header:
    """primary/src/messages.rs:13-21."""

    __slots__ = ("author", "round", "payload", "parents", "id", "signature")

    def __init__(self, author: bytes, round_: int, payload: Optional[Dict[bytes, int]] = None,
                 parents: Optional[Iterable[bytes]] = None, id_: bytes = bytes(32), signature: bytes = bytes(64)):
        self.author = bytes(author)
        self.round = int(round_)
        self.payload = dict(payload or {})
        self.parents = set(bytes(p) for p in (parents or ()))
        self.id = bytes(id_)
        self.signature = bytes(signature)

    def digest_preimage(self) -> bytes:
        """Hash for Header (:70-84): author || round || (digest || worker_id)* || parents*,
        in BTreeMap / BTreeSet (byte) order."""
        parts = [self.author, struct.pack("<Q", self.round)]
        for d in sorted(self.payload):
            parts.append(d + struct.pack("<I", self.payload[d]))
        parts.extend(sorted(self.parents))
        return b"".join(parts)

    def digest(self, engine=None) -> bytes:
        return (engine or _lib.default_engine()).sha512(self.digest_preimage())[:32]

    def to_bytes(self) -> bytes:
        out = [_pk_bytes(self.author), struct.pack("<QQ", self.round, len(self.payload))]
        for d in sorted(self.payload):
            out.append(d + struct.pack("<I", self.payload[d]))
        out.append(struct.pack("<Q", len(self.parents)))
        out.extend(sorted(self.parents))
        out.append(self.id + self.signature)
        return b"".join(out)

    @classmethod
    def read(cls, r: _Reader) -> "Header":
        author = r.public_key()
        round_ = r.u64()
        payload = {}
        for _ in range(r.u64()):
            d = r.take(32)
            payload[d] = r.u32()
        parents = [r.take(32) for _ in range(r.u64())]
        return cls(author, round_, payload, parents, r.take(32), r.take(64))

    def verify(self, committee: Committee, engine=None) -> None:
        """Header::verify (:48-67): id, author stake, worker ids, then the strict signature."""
        eng = engine or _lib.default_engine()
        if self.digest(eng) != self.id:
            raise InvalidHeaderId()
        if committee.stake(self.author) <= 0:
            raise UnknownAuthority(self.author.hex())
        for wid in self.payload.values():
            if not committee.has_worker(self.author, wid):
                raise MalformedHeader(self.id.hex())
        if not eng.verify_strict(self.id, self.author, self.signature):
            raise InvalidSignature()


class Vote:
    """primary/src/messages.rs:105-153."""

    __slots__ = ("id", "round", "origin", "author", "signature")

    def __init__(self, id_: bytes, round_: int, origin: bytes, author: bytes, signature: bytes = bytes(64)):
        self.id = bytes(id_)
        self.round = int(round_)
        self.origin = bytes(origin)
        self.author = bytes(author)
        self.signature = bytes(signature)

    def digest_preimage(self) -> bytes:
        return self.id + struct.pack("<Q", self.round) + self.origin

    def digest(self, engine=None) -> bytes:
        return (engine or _lib.default_engine()).sha512(self.digest_preimage())[:32]

    def to_bytes(self) -> bytes:
        return self.id + struct.pack("<Q", self.round) + _pk_bytes(self.origin) + _pk_bytes(self.author) + self.signature

    @classmethod
    def read(cls, r: _Reader) -> "Vote":
        id_ = r.take(32)
        round_ = r.u64()
        origin = r.public_key()
        author = r.public_key()
        return cls(id_, round_, origin, author, r.take(64))

    def verify(self, committee: Committee, engine=None) -> None:
        """Vote::verify (:131-142)."""
        eng = engine or _lib.default_engine()
        if committee.stake(self.author) <= 0:
            raise UnknownAuthority(self.author.hex())
        if not eng.verify_strict(self.digest(eng), self.author, self.signature):
            raise InvalidSignature()


class Certificate:
    """primary/src/messages.rs:168-256."""

    __slots__ = ("header", "votes")

    def __init__(self, header: Header, votes: Sequence[Tuple[bytes, bytes]] = ()):
        self.header = header
        self.votes = [(bytes(k), bytes(s)) for k, s in votes]

    @staticmethod
    def genesis(committee: Committee) -> List["Certificate"]:
        return [Certificate(Header(name, 0)) for name in committee.keys()]

    def round(self) -> int:
        return self.header.round

    def origin(self) -> bytes:
        return self.header.author

    def is_genesis(self, committee: Committee) -> bool:
        """Certificate::genesis(committee).contains(self) with PartialEq (:249-256): same header id,
        round and origin as a genesis certificate."""
        return self.header.id == bytes(32) and self.round() == 0 and self.origin() in committee.authorities

    def digest_preimage(self) -> bytes:
        """Hash for Certificate (:226-234): header.id || round || origin."""
        return self.header.id + struct.pack("<Q", self.round()) + self.origin()

    def digest(self, engine=None) -> bytes:
        return (engine or _lib.default_engine()).sha512(self.digest_preimage())[:32]

    def to_bytes(self) -> bytes:
        out = [self.header.to_bytes(), struct.pack("<Q", len(self.votes))]
        for k, s in self.votes:
            out.append(_pk_bytes(k) + s)
        return b"".join(out)

    @classmethod
    def read(cls, r: _Reader) -> "Certificate":
        header = Header.read(r)
        votes = []
        for _ in range(r.u64()):
            k = r.public_key()
            votes.append((k, r.take(64)))
        return cls(header, votes)

    def _quorum(self, committee: Committee) -> None:
        weight = 0
        used = set()
        for name, _ in self.votes:
            if name in used:
                raise AuthorityReuse(name.hex())
            st = committee.stake(name)
            if st <= 0:
                raise UnknownAuthority(name.hex())
            used.add(name)
            weight += st
        if weight < committee.quorum_threshold():
            raise CertificateRequiresQuorum()

    def verify(self, committee: Committee, engine=None, zseed: Optional[bytes] = None) -> None:
        """Certificate::verify (:189-215)."""
        errs = verify_certificates([self], committee, engine, zseed)
        if errs[0] is not None:
            raise errs[0]


# PrimaryMessage (primary/src/primary.rs:33-38): variant index u32
_VARIANTS = {0: Header, 1: Vote, 2: Certificate}


def encode_primary_message(msg) -> bytes:
    for tag, cls in _VARIANTS.items():
        if isinstance(msg, cls):
            return struct.pack("<I", tag) + msg.to_bytes()
    raise TypeError("not a PrimaryMessage variant: %r" % (msg,))


def decode_primary_message(buf: bytes):
    r = _Reader(buf)
    tag = r.u32()
    if tag not in _VARIANTS:
        raise SerializationError("unsupported PrimaryMessage variant %d" % tag)
    # bincode::deserialize (bincode 1.3, primary/src/primary.rs:236) allows trailing bytes
    return _VARIANTS[tag].read(r)


# ----------------------------------------------------------------------------- bulk (Core batching)
class _CommitteeSlots:
    """Committee keys loaded once into an engine's key cache (nw_committee_load)."""

    def __init__(self, engine, committee: Committee):
        keys = committee.keys()
        self.slots = dict(zip(keys, engine.committee_load(keys, [committee.stake(k) for k in keys])))


_slot_cache: Dict[Tuple[int, Tuple[bytes, ...]], _CommitteeSlots] = {}


def committee_slots(engine, committee: Committee) -> Dict[bytes, int]:
    key = (id(engine), tuple(committee.keys()))
    cs = _slot_cache.get(key)
    if cs is None:
        cs = _slot_cache[key] = _CommitteeSlots(engine, committee)
    return cs.slots


def verify_certificates(certs: Sequence[Certificate], committee: Committee, engine=None,
                        zseed: Optional[bytes] = None, cert_base: int = 0) -> List[Optional[DagError]]:
    """``Certificate::verify`` for many certificates: returns, per certificate, None (Ok) or the
    DagError the reference would return, checked in the reference's order.  GPU submissions: one
    SHA-512 batch for every header and certificate digest, one strict verify batch for the header
    signatures, one certificate batch verify (nw_verify_certs) for the votes."""
    import os
    eng = engine or _lib.default_engine()
    n = len(certs)
    out: List[Optional[DagError]] = [None] * n
    if n == 0:
        return out
    if zseed is None:
        zseed = os.urandom(32)
    todo = [i for i, c in enumerate(certs) if not c.is_genesis(committee)]
    # digests: header ids and certificate digests in one GPU submission
    pre = [certs[i].header.digest_preimage() for i in todo] + [certs[i].digest_preimage() for i in todo]
    dig = eng.sha512_many(pre)
    hdr_digest = {i: dig[k][:32] for k, i in enumerate(todo)}
    cert_digest = {i: dig[len(todo) + k][:32] for k, i in enumerate(todo)}
    # Header::verify up to its signature
    live = []
    for i in todo:
        h = certs[i].header
        if hdr_digest[i] != h.id:
            out[i] = InvalidHeaderId()
        elif committee.stake(h.author) <= 0:
            out[i] = UnknownAuthority(h.author.hex())
        elif any(not committee.has_worker(h.author, w) for w in h.payload.values()):
            out[i] = MalformedHeader(h.id.hex())
        else:
            live.append(i)
    # header signatures: one strict-verify submission (committee keys cached first: comb path)
    if live:
        committee_slots(eng, committee)
        ok = eng.verify_strict_many([certs[i].header.id for i in live], [certs[i].header.author for i in live],
                                    [certs[i].header.signature for i in live])
        nxt = []
        for i, good in zip(live, ok):
            if not good:
                out[i] = InvalidSignature()
            else:
                nxt.append(i)
        live = nxt
    # quorum checks (host), then one batch-verify submission over every remaining certificate
    ready = []
    for i in live:
        try:
            certs[i]._quorum(committee)
            ready.append(i)
        except DagError as e:
            out[i] = e
    if ready:
        slots = committee_slots(eng, committee)
        ranges, signer, sigs, msgs = [], [], [], []
        for i in ready:
            ranges.append((len(signer), len(certs[i].votes)))
            for k, s in certs[i].votes:
                signer.append(slots[k])
                sigs.append(s)
            msgs.append(cert_digest[i])
        cert_ok, _, _ = eng.verify_certs(ranges, b"".join(sigs), signer, b"".join(msgs), zseed,
                                         cert_base=cert_base)
        for i, good in zip(ready, cert_ok):
            if not good:
                out[i] = InvalidSignature()
    return out


# ----------------------------------------------------------------------------- native wire path
class NotACertificate(DagError):
    """A well-formed PrimaryMessage that is not a Certificate (the native certificate path only)."""


_DAG_KIND = {
    _lib.DAG_INVALID_SIGNATURE: InvalidSignature, _lib.DAG_SERIALIZATION: SerializationError,
    _lib.DAG_INVALID_HEADER_ID: InvalidHeaderId, _lib.DAG_MALFORMED_HEADER: MalformedHeader,
    _lib.DAG_UNKNOWN_AUTHORITY: UnknownAuthority, _lib.DAG_AUTHORITY_REUSE: AuthorityReuse,
    _lib.DAG_REQUIRES_QUORUM: CertificateRequiresQuorum, _lib.DAG_NOT_CERTIFICATE: NotACertificate,
}

_abi_cache: Dict[int, Tuple[Committee, "_lib.CommitteeABI"]] = {}


def committee_abi(committee: Committee) -> "_lib.CommitteeABI":
    """nw_committee view of a Committee (BTreeMap order, as nw_committee_load gets it)."""
    hit = _abi_cache.get(id(committee))
    if hit is None or hit[0] is not committee:
        keys = committee.keys()
        abi = _lib.CommitteeABI(keys, [committee.stake(k) for k in keys],
                                [committee.authorities[k][1] for k in keys])
        hit = _abi_cache[id(committee)] = (committee, abi)
    return hit[1]


def decode_certificate_frames(frames: Sequence[bytes], committee: Committee) -> "_lib.CertBatch":
    """Native (C++) bincode decode + host checks of many PrimaryMessage frames (no GPU)."""
    return _lib.CertBatch(committee_abi(committee), frames)


def verify_certificate_frames(frames: Sequence[bytes], committee: Committee, engine=None,
                              zseed: Optional[bytes] = None, cert_base: int = 0) -> List[Optional[DagError]]:
    """What the primary does with each received ``PrimaryMessage::Certificate`` frame
    (primary/src/primary.rs:236 deserialize, then Certificate::verify, messages.rs:189-215), for many
    frames at once on the native path: C++ decode into SoA, then three GPU submissions.  Returns
    None (Ok) or the DagError per frame; same verdicts and coefficient indexing as
    ``verify_certificates`` over the decoded certificates."""
    import os
    eng = engine or _lib.default_engine()
    if zseed is None:
        zseed = os.urandom(32)
    batch = decode_certificate_frames(frames, committee)
    try:
        codes = eng.cert_batch_verify(batch, zseed, cert_base)
    finally:
        batch.close()
    return [None if c == _lib.DAG_OK else _DAG_KIND[c]() for c in codes]
