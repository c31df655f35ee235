"""CPU oracle for the Ed25519 verify + SHA-512 hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker* the HIP path is compared against.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may import it;
nothing in ``narwhal_amd/`` may (the product fails loudly when its HIP library is absent).

What it restates
----------------
The reference's hot path lives in third-party Rust crates that are NOT vendored under
/root/reference and have no Cargo.lock:

* ``ed25519-dalek 1.0.1`` with ``features=["batch"]``   (crypto/Cargo.toml:10)
* ``curve25519-dalek 3.x`` (u64 backend)                  (transitive)
* ``ed25519 1.x``  (``Signature::from_bytes`` high-bit check)
* ``sha2 0.9``     (``Sha512`` = FIPS 180-4)              (re-exported as ed25519_dalek::Sha512)
* ``merlin 2`` + ``rand 0.7`` ``thread_rng`` (batch coefficients; non-deterministic)

Their published algorithms are restated here with Python integers.  The reference call
sites each function follows are cited in its docstring.  Where the reference draws batch
coefficients from ``thread_rng`` (unreproducible), this oracle takes the coefficients ``z``
as an explicit input; the product and the oracle derive them from the same seeded
ChaCha20 stream (``batch_coefficients``), so verdicts are comparable bit for bit.

Pinning (see tests/test_oracle_golden.py and tests/golden/README.md):
* RFC 8032 §7.1 TEST 1 (published known answer), cross-checked against libsodium 1.0.18
  (independent implementation, available only in the build container);
* the reference's deterministic fixtures: ``keys()`` = 4 dalek keypairs from
  ``StdRng::from_seed([0;32])`` (crypto/src/tests/crypto_tests.rs:26-29,
  primary/src/tests/common.rs:29-32) = ChaCha20 zero-key keystream, and the worker batch
  digest fixture (worker/src/tests/common.rs:92-109);
* the reference's own test verdicts (crypto/src/tests/crypto_tests.rs:49-115).
Adversarial semantics (small order, non-canonical, torsion) are not covered by any
reference fixture: those vectors are "parity unpinned" w.r.t. the reference and are
pinned only by this restatement of the published crate semantics.
"""
from __future__ import annotations

import hashlib
import struct
from typing import List, Optional, Sequence, Tuple

# ----------------------------------------------------------------------------- constants
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)
BASE_Y = (4 * pow(5, P - 2, P)) % P


def _recover_base() -> Tuple[int, int, int, int]:
    y = BASE_Y
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    assert ok and x % 2 == 0
    return (x, y, 1, x * y % P)


# ----------------------------------------------------------------------------- field
def fe_is_negative(x: int) -> bool:
    """curve25519-dalek FieldElement::is_negative: low bit of the canonical encoding."""
    return (x % P) & 1 == 1


def sqrt_ratio_i(u: int, v: int) -> Tuple[bool, int]:
    """curve25519-dalek 3.x ``FieldElement::sqrt_ratio_i`` [dalek-spec].

    Returns (was_nonzero_square, r) with r the *nonnegative* root of u/v (or of i*u/v).
    u == 0 yields (True, 0).  Reached from ``CompressedEdwardsY::decompress`` which
    ``dalek::PublicKey::from_bytes`` (crypto/src/lib.rs:186,202,216) and the R decoding
    in ``verify_strict``/``verify_batch`` call.
    """
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = (u * v3 % P) * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u) * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    if fe_is_negative(r):
        r = (-r) % P
    return (correct or flipped), r


# ----------------------------------------------------------------------------- points
# Extended twisted-Edwards coordinates (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z, a = -1.
IDENTITY = (0, 1, 1, 0)


def pt_add(p1, p2):
    """Complete unified addition (Hisil-Wong-Carter-Dawson 2008, a = -1)."""
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    Bv = (Y1 + X1) * (Y2 + X2) % P
    C = 2 * D * T1 * T2 % P
    Dd = 2 * Z1 * Z2 % P
    E, F, G, H = Bv - A, Dd - C, Dd + C, Bv + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def pt_neg(p1):
    X, Y, Z, T = p1
    return ((-X) % P, Y, Z, (-T) % P)


def pt_double(p1):
    return pt_add(p1, p1)


def pt_mul(k: int, p1):
    """Exact integer multiple k*P (k >= 0), plain double-and-add (vartime is fine here)."""
    assert k >= 0
    acc = IDENTITY
    q = p1
    while k:
        if k & 1:
            acc = pt_add(acc, q)
        q = pt_double(q)
        k >>= 1
    return acc


def pt_eq(p1, p2) -> bool:
    """curve25519-dalek ``EdwardsPoint::ct_eq``: projective equality X1 Z2 == X2 Z1, Y1 Z2 == Y2 Z1."""
    X1, Y1, Z1, _ = p1
    X2, Y2, Z2, _ = p2
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def pt_is_identity(p1) -> bool:
    """``EdwardsPoint::is_identity`` (compress() == identity encoding)."""
    return pt_eq(p1, IDENTITY)


def pt_is_small_order(p1) -> bool:
    """``EdwardsPoint::is_small_order``: [8]P == identity."""
    return pt_is_identity(pt_mul(8, p1))


def pt_compress(p1) -> bytes:
    X, Y, Z, _ = p1
    zi = pow(Z, P - 2, P)
    x, y = X * zi % P, Y * zi % P
    return ((y | ((x & 1) << 255))).to_bytes(32, "little")


B_POINT = _recover_base()


def decompress(b: bytes) -> Optional[tuple]:
    """curve25519-dalek 3.x ``CompressedEdwardsY::decompress`` [dalek-spec].

    * y = bytes with bit 255 cleared, taken mod p WITHOUT rejecting y >= p
      (``FieldElement::from_bytes``);
    * u = y^2 - 1, v = d y^2 + 1; ``sqrt_ratio_i`` failure -> None;
    * x = nonnegative root, negated when bit 255 is set (x = 0 with the sign bit set is
      accepted and stays 0).
    Called per vote by ``dalek::PublicKey::from_bytes`` (crypto/src/lib.rs:216) and for R.
    """
    assert len(b) == 32
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    y %= P
    yy = y * y % P
    u = (yy - 1) % P
    v = (D * yy + 1) % P
    ok, x = sqrt_ratio_i(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P
    return (x, y, 1, x * y % P)


# ----------------------------------------------------------------------------- scalars / hashes
def sha512(data: bytes) -> bytes:
    """sha2 0.9 ``Sha512`` (FIPS 180-4) — ``ed25519_dalek::Sha512`` at primary/src/messages.rs:72,147,228,
    worker/src/processor.rs:65, worker/src/batch_maker.rs:125."""
    return hashlib.sha512(data).digest()


def digest32(data: bytes) -> bytes:
    """The reference's ``Digest`` = SHA-512 truncated to 32 bytes (e.g. crypto_tests.rs:8-12)."""
    return sha512(data)[:32]


def scalar_from_hash(h64: bytes) -> int:
    """curve25519-dalek ``Scalar::from_hash`` = 64-byte LE integer mod l."""
    return int.from_bytes(h64, "little") % L


def sig_parse(sig: bytes) -> Optional[Tuple[bytes, int]]:
    """Signature parsing on every reference path.

    1. ``ed25519::Signature::from_bytes`` (crypto/src/lib.rs:201,215): Err when
       ``S[31] & 0xE0 != 0``.
    2. dalek ``InternalSignature::try_from`` -> ``check_scalar`` (default features, no
       ``legacy_compatibility``): when the top 4 bits of S are clear it succeeds fast,
       otherwise ``Scalar::from_canonical_bytes`` (S < l) must succeed.
    Net effect: Ok iff S < l.  R stays raw bytes.
    """
    assert len(sig) == 64
    R, Sb = sig[:32], sig[32:]
    if Sb[31] & 0xE0:
        return None
    s = int.from_bytes(Sb, "little")
    if Sb[31] & 0xF0 and s >= L:
        return None
    return R, s


# ----------------------------------------------------------------------------- verification
def verify_strict(pk: bytes, msg: bytes, sig: bytes) -> bool:
    """``crypto::Signature::verify`` (crypto/src/lib.rs:200-204) =
    ed25519::Signature::from_bytes -> dalek::PublicKey::from_bytes -> ``verify_strict``.

    dalek 1.0.1 ``PublicKey::verify_strict`` [dalek-spec]: decompress R (fail -> Err);
    Err if R or A is small order; k = from_hash(SHA512(R_bytes || A_bytes || M));
    R' = k(-A) + sB; Ok iff R' == R as projective points.
    """
    parsed = sig_parse(sig)
    if parsed is None:
        return False
    Rb, s = parsed
    A = decompress(pk)
    if A is None:
        return False
    R = decompress(Rb)
    if R is None:
        return False
    if pt_is_small_order(R) or pt_is_small_order(A):
        return False
    k = scalar_from_hash(sha512(Rb + pk + msg))
    Rp = pt_add(pt_mul(k, pt_neg(A)), pt_mul(s, B_POINT))
    return pt_eq(Rp, R)


def verify_batch_z(msgs: Sequence[bytes], sigs: Sequence[bytes], pks: Sequence[bytes],
                   zs: Sequence[int]) -> bool:
    """dalek 1.0.1 ``verify_batch`` with the 128-bit coefficients ``zs`` supplied [dalek-spec].

    Called from crypto/src/lib.rs:218 (certificates) and worker/src/processor.rs:78.
    * length mismatch -> Err;
    * every S parsed (``InternalSignature::try_from``; any failure -> Err);
    * h_i = from_hash(SHA512(R_i || A_i || M_i)) (raw R and A bytes);
    * B_coef = sum z_i s_i mod l ; zh_i = z_i h_i mod l;
    * id = (-B_coef) B + sum z_i R_i + sum zh_i A_i  (R_i decompress failure -> Err);
    * Ok iff id is the identity: cofactorless, no small-order rejection.
    ``pks`` must already be decodable (the caller's ``PublicKey::from_bytes`` succeeded).
    """
    n = len(sigs)
    if len(msgs) != n or len(pks) != n or len(zs) != n:
        return False
    parsed = [sig_parse(s) for s in sigs]
    if any(p is None for p in parsed):
        return False
    As = [decompress(pk) for pk in pks]
    if any(a is None for a in As):
        return False
    hs = [scalar_from_hash(sha512(parsed[i][0] + pks[i] + msgs[i])) for i in range(n)]
    bcoef = sum(zs[i] * parsed[i][1] for i in range(n)) % L
    acc = pt_mul((-bcoef) % L, B_POINT)
    for i in range(n):
        R = decompress(parsed[i][0])
        if R is None:
            return False
        acc = pt_add(acc, pt_mul(zs[i], R))
        acc = pt_add(acc, pt_mul(zs[i] * hs[i] % L, As[i]))
    return pt_is_identity(acc)


# ----------------------------------------------------------------------------- seeded coefficients
def _rotl32(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


def chacha20_block(key: bytes, counter: int, nonce: bytes, rounds: int = 20) -> bytes:
    """RFC 8439 §2.3 ChaCha20 block function (32-bit counter, 96-bit nonce)."""
    assert len(key) == 32 and len(nonce) == 12
    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    st += list(struct.unpack("<8I", key))
    st += [counter & 0xFFFFFFFF]
    st += list(struct.unpack("<3I", nonce))
    w = list(st)

    def qr(a, b, c, d):
        w[a] = (w[a] + w[b]) & 0xFFFFFFFF; w[d] = _rotl32(w[d] ^ w[a], 16)
        w[c] = (w[c] + w[d]) & 0xFFFFFFFF; w[b] = _rotl32(w[b] ^ w[c], 12)
        w[a] = (w[a] + w[b]) & 0xFFFFFFFF; w[d] = _rotl32(w[d] ^ w[a], 8)
        w[c] = (w[c] + w[d]) & 0xFFFFFFFF; w[b] = _rotl32(w[b] ^ w[c], 7)

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return struct.pack("<16I", *[(w[i] + st[i]) & 0xFFFFFFFF for i in range(16)])


def chacha20_stream(key: bytes, nbytes: int, nonce: bytes = b"\0" * 12) -> bytes:
    out = b""
    ctr = 0
    while len(out) < nbytes:
        out += chacha20_block(key, ctr, nonce)
        ctr += 1
    return out[:nbytes]


def batch_coefficients(zseed: bytes, batch_index: int, n: int) -> List[int]:
    """Seeded replacement for dalek's merlin/thread_rng coefficients (SURVEY.md §7 hard part 2).

    NW-Z v1:  z_i = LE-u128( ChaCha20(key = zseed, counter = i,
                                       nonce = u32le(batch_index_lo) || u32le(batch_index_hi) || 0)[0:16] ).
    Each certificate (``batch_index``) draws from its own stream, so shards need no exchange.
    """
    nonce = struct.pack("<III", batch_index & 0xFFFFFFFF, (batch_index >> 32) & 0xFFFFFFFF, 0)
    return [int.from_bytes(chacha20_block(zseed, i, nonce)[:16], "little") for i in range(n)]


def crypto_verify_batch(digest: bytes, votes: Sequence[Tuple[bytes, bytes]], zseed: bytes,
                        batch_index: int = 0) -> bool:
    """``crypto::Signature::verify_batch`` (crypto/src/lib.rs:206-219): per vote, in order,
    ``ed25519::Signature::from_bytes`` (S top-3-bit check) and ``dalek::PublicKey::from_bytes``
    with early ``?`` return, then ``dalek::verify_batch`` with ``[digest; n]``."""
    for pk, sig in votes:
        if sig[63] & 0xE0:
            return False
        if decompress(pk) is None:
            return False
    n = len(votes)
    zs = batch_coefficients(zseed, batch_index, n)
    return verify_batch_z([digest] * n, [s for _, s in votes], [k for k, _ in votes], zs)


# ----------------------------------------------------------------------------- signing (fixtures only)
def expand_secret(seed: bytes) -> Tuple[int, bytes]:
    h = sha512(seed)
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(bytes(a), "little"), h[32:]


def public_from_seed(seed: bytes) -> bytes:
    """dalek ``PublicKey::from(&SecretKey)`` (RFC 8032 §5.1.5)."""
    a, _ = expand_secret(seed)
    return pt_compress(pt_mul(a, B_POINT))


def sign(seed: bytes, msg: bytes) -> bytes:
    """RFC 8032 Ed25519 signing = dalek ``Keypair::sign`` used by ``crypto::Signature::new``
    (crypto/src/lib.rs:185-191).  Used only to make fixtures."""
    a, prefix = expand_secret(seed)
    A = pt_compress(pt_mul(a, B_POINT))
    r = scalar_from_hash(sha512(prefix + msg))
    Rb = pt_compress(pt_mul(r, B_POINT))
    k = scalar_from_hash(sha512(Rb + A + msg))
    s = (r + k * a) % L
    return Rb + s.to_bytes(32, "little")


def reference_fixture_seeds(n: int = 4) -> List[bytes]:
    """``keys()`` fixture: ``StdRng::from_seed([0;32])`` (rand 0.7 StdRng = ChaCha20Rng,
    key = seed, nonce/counter = 0) feeding ``SecretKey::generate`` (``fill_bytes`` of 32 B)
    n times (crypto/src/tests/crypto_tests.rs:26-29, primary/src/tests/common.rs:29-32)."""
    ks = chacha20_stream(b"\0" * 32, 32 * n)
    return [ks[32 * i:32 * (i + 1)] for i in range(n)]


# ----------------------------------------------------------------------------- reference message formats
def bincode_worker_batch(txs: Sequence[bytes]) -> bytes:
    """bincode 1.x of ``WorkerMessage::Batch(Vec<Vec<u8>>)`` (worker/src/worker.rs:36-39,
    worker/src/batch_maker.rs:118-119): u32 variant 0, u64 count, then (u64 len, bytes)*."""
    out = [struct.pack("<IQ", 0, len(txs))]
    for t in txs:
        out.append(struct.pack("<Q", len(t)))
        out.append(bytes(t))
    return b"".join(out)


def header_digest(author: bytes, round_: int, payload: Sequence[Tuple[bytes, int]],
                  parents: Sequence[bytes]) -> bytes:
    """``impl Hash for Header`` (primary/src/messages.rs:70-84): BTreeMap/BTreeSet order."""
    h = hashlib.sha512()
    h.update(author)
    h.update(struct.pack("<Q", round_))
    for x, y in sorted(payload):
        h.update(x)
        h.update(struct.pack("<I", y))
    for x in sorted(parents):
        h.update(x)
    return h.digest()[:32]


def vote_digest(header_id: bytes, round_: int, origin: bytes) -> bytes:
    """``impl Hash for Vote`` / ``impl Hash for Certificate`` (primary/src/messages.rs:145-153,226-234)."""
    return digest32(header_id + struct.pack("<Q", round_) + origin)


# ----------------------------------------------------------------------------- torsion helpers (vectors)
def small_order_points() -> List[tuple]:
    """The 8 points of order dividing 8."""
    # an order-8 point: decompress a y that gives order 8
    pts = []
    seen = set()
    # generate E[8] as 5 * l * P for a few decodable P
    for t in range(2, 200):
        Pp = decompress(t.to_bytes(32, "little"))
        if Pp is None:
            continue
        T = pt_mul(5 * L, Pp)  # torsion component of Pp (l = 5 mod 8, 5*5 = 1 mod 8)
        for k in range(8):
            Q = pt_mul(k, T)
            enc = pt_compress(Q)
            if enc not in seen:
                seen.add(enc)
                pts.append(Q)
        if len(pts) == 8:
            break
    return pts


def small_order_generator() -> tuple:
    """The generator T8 of E[8] used by the device code (tools/gen_constants.py): the first point
    of ``small_order_points()`` of exact order 8."""
    for q in small_order_points():
        if not pt_is_identity(pt_mul(4, q)):
            return q
    raise AssertionError("no order-8 point")
