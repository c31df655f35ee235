"""Deterministic honest and adversarial Ed25519 vectors built from the oracle's primitives.

Classes follow SURVEY.md §8(c): (i) small-order A, (ii) R = identity, (iii) mixed-order R,
(iv) mixed-order A, (v) S >= l, (vi) S with high bits, (vii) undecodable R / A,
(viii) non-canonical encodings, (ix) wrong message / key, plus a crafted pair of invalid
signatures whose residuals cancel in the batch equation for one known coefficient stream
(exercises the exactness of the batch path, not just its honest case).
The expected verdicts always come from the oracle (``verify_strict`` / ``verify_batch_z``).
"""
from __future__ import annotations

import os
import random
import sys
from typing import List, Tuple

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import ed25519_oracle as o  # noqa: E402

Case = Tuple[str, bytes, bytes, bytes]   # (name, pk, sig, msg)
P, L = o.P, o.L


def _rand_bytes(rng: random.Random, n: int) -> bytes:
    return bytes(rng.randrange(256) for _ in range(n))


def _sign_raw(a: int, A_bytes: bytes, r: int, msg: bytes, R_point=None, R_bytes: bytes = None) -> bytes:
    """Signature (R, s = r + H(R||A||M) a) with an explicit nonce / R point / R encoding."""
    if R_point is None:
        R_point = o.pt_mul(r, o.B_POINT)
    Rb = R_bytes if R_bytes is not None else o.pt_compress(R_point)
    k = o.scalar_from_hash(o.sha512(Rb + A_bytes + msg))
    s = (r + k * a) % L
    return Rb + s.to_bytes(32, "little")


def honest_cases(rng: random.Random, n: int, msg_len: int = 32) -> List[Case]:
    out = []
    for i in range(n):
        seed = _rand_bytes(rng, 32)
        msg = _rand_bytes(rng, msg_len)
        out.append(("honest%d" % i, o.public_from_seed(seed), o.sign(seed, msg), msg))
    return out


def noncanonical_encodings() -> List[bytes]:
    """y >= p encodings (y + p < 2^255 for y in 0..18), with and without the sign bit."""
    out = []
    for y in range(19):
        for sign in (0, 1):
            out.append(((y + P) | (sign << 255)).to_bytes(32, "little"))
    return out


def undecodable_encoding(rng: random.Random) -> bytes:
    while True:
        b = _rand_bytes(rng, 32)
        if o.decompress(b) is None:
            return b


def adversarial_cases(rng: random.Random) -> List[Case]:
    cases: List[Case] = []
    msg = _rand_bytes(rng, 32)
    small = o.small_order_points()
    T8 = o.small_order_generator()
    # (i) small-order A (canonical encodings of all 8, plus non-canonical identity / order-2 forms)
    small_encs = [o.pt_compress(t) for t in small]
    small_encs += [(1 + P).to_bytes(32, "little"), ((1 + P) | (1 << 255)).to_bytes(32, "little"),
                   (1 | (1 << 255)).to_bytes(32, "little")]
    for j, Ab in enumerate(small_encs):
        if o.decompress(Ab) is None:
            continue
        r = rng.randrange(1, L)
        Rp = o.pt_mul(r, o.B_POINT)
        cases.append(("i_smallA_%d" % j, Ab, o.pt_compress(Rp) + r.to_bytes(32, "little"), msg))
    # (ii) R = identity, S = k a (and the x=0 / sign-bit-set identity encoding)
    for j, Rb in enumerate([o.pt_compress(o.IDENTITY), (1 | (1 << 255)).to_bytes(32, "little")]):
        a = rng.randrange(1, L)
        Ab = o.pt_compress(o.pt_mul(a, o.B_POINT))
        k = o.scalar_from_hash(o.sha512(Rb + Ab + msg))
        cases.append(("ii_Rident_%d" % j, Ab, Rb + (k * a % L).to_bytes(32, "little"), msg))
    # (iii) mixed-order R = rB + T  (several torsion orders)
    for j, mult in enumerate([1, 2, 4, 3]):
        a = rng.randrange(1, L)
        Ab = o.pt_compress(o.pt_mul(a, o.B_POINT))
        r = rng.randrange(1, L)
        Rp = o.pt_add(o.pt_mul(r, o.B_POINT), o.pt_mul(mult, T8))
        cases.append(("iii_mixedR_%d" % j, Ab, _sign_raw(a, Ab, r, msg, R_point=Rp), msg))
    # (iv) mixed-order A = aB + T
    for j, mult in enumerate([1, 2, 4, 5, 6, 7]):
        a = rng.randrange(1, L)
        A = o.pt_add(o.pt_mul(a, o.B_POINT), o.pt_mul(mult, T8))
        Ab = o.pt_compress(A)
        for t in range(3):
            r = rng.randrange(1, L)
            cases.append(("iv_mixedA_%d_%d" % (j, t), Ab, _sign_raw(a, Ab, r, msg), msg))
    # honest base for malleations
    seed = _rand_bytes(rng, 32)
    pk = o.public_from_seed(seed)
    sig = o.sign(seed, msg)
    s = int.from_bytes(sig[32:], "little")
    # (v) S >= l
    for j, s2 in enumerate([s + L, L, L + 1]):
        if s2 < 2**256:
            cases.append(("v_Sbig_%d" % j, pk, sig[:32] + s2.to_bytes(32, "little"), msg))
    # (vi) high bits of S
    for j, bit in enumerate([253, 254, 255]):
        cases.append(("vi_Shigh_%d" % j, pk, sig[:32] + (s | (1 << bit)).to_bytes(32, "little"), msg))
    # (vii) undecodable R / A
    cases.append(("vii_badR", pk, undecodable_encoding(rng) + sig[32:], msg))
    cases.append(("vii_badA", undecodable_encoding(rng), sig, msg))
    # (viii) non-canonical encodings as R and as A
    for j, e in enumerate(noncanonical_encodings()):
        if o.decompress(e) is None:
            continue
        cases.append(("viii_ncR_%d" % j, pk, e + sig[32:], msg))
        cases.append(("viii_ncA_%d" % j, e, sig, msg))
    # non-canonical R encoding of a point whose discrete log we know is impossible (y < 19 points
    # have unknown logs), so use R = identity non-canonically with S = k a: strict rejects (small)
    a = rng.randrange(1, L)
    Ab = o.pt_compress(o.pt_mul(a, o.B_POINT))
    Rb = (1 + P).to_bytes(32, "little")
    k = o.scalar_from_hash(o.sha512(Rb + Ab + msg))
    cases.append(("viii_ncRident", Ab, Rb + (k * a % L).to_bytes(32, "little"), msg))
    # (ix) wrong message / wrong key / S = 0 default signature
    cases.append(("ix_wrongmsg", pk, sig, o.digest32(b"Bad message!")))
    cases.append(("ix_wrongkey", o.public_from_seed(_rand_bytes(rng, 32)), sig, msg))
    cases.append(("ix_zero_sig", pk, bytes(64), msg))
    cases.append(("honest_ref", pk, sig, msg))
    return cases


def cancelling_pair(zseed: bytes, bidx: int, rng: random.Random, n_honest: int = 2):
    """Batch (pk, sig, msg) list with two INVALID signatures whose residuals D_1, D_2 satisfy
    z_1 D_1 + z_2 D_2 = O for the NW-Z v1 stream (zseed, bidx): dalek's batch equation accepts
    it while both strict verdicts reject.  Positions: the invalid pair is last."""
    items = []
    for h in honest_cases(rng, n_honest):
        items.append((h[1], h[2], h[3]))
    n = len(items) + 2
    zs = o.batch_coefficients(zseed, bidx, n)
    z1, z2 = zs[-2], zs[-1]
    msg = _rand_bytes(rng, 32)
    # sig 1: D_1 = d1 B
    a1 = rng.randrange(1, L)
    A1 = o.pt_compress(o.pt_mul(a1, o.B_POINT))
    r1 = rng.randrange(1, L)
    R1 = o.pt_compress(o.pt_mul(r1, o.B_POINT))
    k1 = o.scalar_from_hash(o.sha512(R1 + A1 + msg))
    d1 = rng.randrange(1, L)
    s1 = (r1 + k1 * a1 - d1) % L           # D_1 = R1 + k1 A1 - s1 B = d1 B
    # sig 2: D_2 = c d1 B with c = -z1 / z2 mod l
    c = (-z1 * pow(z2, L - 2, L)) % L
    a2 = rng.randrange(1, L)
    A2 = o.pt_compress(o.pt_mul(a2, o.B_POINT))
    r2 = rng.randrange(1, L)
    R2 = o.pt_compress(o.pt_mul(r2, o.B_POINT))
    k2 = o.scalar_from_hash(o.sha512(R2 + A2 + msg))
    s2 = (r2 + k2 * a2 - c * d1) % L
    items.append((A1, R1 + s1.to_bytes(32, "little"), msg))
    items.append((A2, R2 + s2.to_bytes(32, "little"), msg))
    return items
