"""GPU: the primary-side callers of the hot path (narwhal_amd.primary) — Header::verify,
Vote::verify, Certificate::verify (primary/src/messages.rs:48-67,131-142,189-215) with the
reference's fixtures (primary/src/tests/common.rs:96-166) and its error kinds, and the bulk
Core-side form verify_certificates against per-certificate verification and the oracle."""
import random

import pytest

import ed25519_oracle as o
from narwhal_amd import primary as pm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world():
    seeds = o.reference_fixture_seeds(4)
    keys = [o.public_from_seed(s) for s in seeds]
    com = pm.Committee({k: (1, [0]) for k in keys})
    return seeds, keys, com


def make_header(seeds, keys, com, author_idx=3, round_=1, payload=None, engine=None):
    parents = [o.digest32(c.digest_preimage()) for c in pm.Certificate.genesis(com)]
    h = pm.Header(keys[author_idx], round_, payload or {}, parents)
    h.id = o.digest32(h.digest_preimage())
    h.signature = o.sign(seeds[author_idx], h.id)
    return h


def make_cert(seeds, keys, com, h, voters=(0, 1, 2, 3)):
    v = pm.Vote(h.id, h.round, h.author, keys[0])
    d = o.digest32(v.digest_preimage())
    return pm.Certificate(h, [(keys[i], o.sign(seeds[i], d)) for i in voters])


def test_reference_fixtures(engine, world, golden):
    seeds, keys, com = world
    h = make_header(seeds, keys, com)
    assert h.id.hex() == golden["primary_fixtures"]["header"]["id"]
    assert h.signature.hex() == golden["primary_fixtures"]["header"]["signature"]
    h.verify(com, engine)
    assert h.digest(engine) == h.id
    for i in range(4):
        v = pm.Vote(h.id, h.round, h.author, keys[i])
        v.signature = o.sign(seeds[i], o.digest32(v.digest_preimage()))
        v.verify(com, engine)
    cert = make_cert(seeds, keys, com, h)
    assert cert.digest(engine).hex() == golden["primary_fixtures"]["certificate_digest"]
    cert.verify(com, engine)
    back = pm.decode_primary_message(pm.encode_primary_message(cert))
    back.verify(com, engine)


def test_error_kinds(engine, world):
    seeds, keys, com = world
    h = make_header(seeds, keys, com)
    good = make_cert(seeds, keys, com, h)
    cases = []
    # genesis: always Ok
    cases.append((pm.Certificate.genesis(com)[1], None))
    # header id mismatch
    bad_id = make_cert(seeds, keys, com, make_header(seeds, keys, com))
    bad_id.header.round = 2
    cases.append((bad_id, pm.InvalidHeaderId))
    # unknown header author (id recomputed so the digest check passes)
    stranger = bytes([9]) * 32
    hs = make_header(seeds, keys, com)
    hs.author = o.public_from_seed(stranger)
    hs.id = o.digest32(hs.digest_preimage())
    hs.signature = o.sign(stranger, hs.id)
    cases.append((pm.Certificate(hs, good.votes), pm.UnknownAuthority))
    # worker id not in the committee -> MalformedHeader
    hm = make_header(seeds, keys, com, payload={bytes([5]) * 32: 7})
    cases.append((make_cert(seeds, keys, com, hm), pm.MalformedHeader))
    # bad header signature
    hb = make_header(seeds, keys, com)
    hb.signature = o.sign(seeds[0], hb.id)
    cases.append((make_cert(seeds, keys, com, hb), pm.InvalidSignature))
    # quorum rules
    cases.append((pm.Certificate(h, good.votes[:2]), pm.CertificateRequiresQuorum))
    cases.append((pm.Certificate(h, good.votes[:2] + good.votes[:1]), pm.AuthorityReuse))
    cases.append((pm.Certificate(h, good.votes[:2] + [(o.public_from_seed(stranger), good.votes[2][1])]),
                  pm.UnknownAuthority))
    # a bad vote signature (the reference's all-zero Signature::default) -> batch Err
    cases.append((pm.Certificate(h, good.votes[:3] + [(keys[3], bytes(64))]), pm.InvalidSignature))
    cases.append((good, None))
    for cert, want in cases:
        if want is None:
            cert.verify(com, engine)
        else:
            with pytest.raises(want):
                cert.verify(com, engine)
    got = pm.verify_certificates([c for c, _ in cases], com, engine)
    assert [type(e) if e else None for e in got] == [w for _, w in cases]
    # the native wire path (C++ bincode decode + the same three GPU submissions) on the frames
    frames = [pm.encode_primary_message(c) for c, _ in cases]
    frames.append(frames[-1][:-3])                                               # truncated
    frames.append(pm.encode_primary_message(pm.Vote(h.id, 1, h.author, keys[0])))  # not a certificate
    native = pm.verify_certificate_frames(frames, com, engine)
    assert [type(e) if e else None for e in native] == [w for _, w in cases] + [pm.SerializationError,
                                                                               pm.NotACertificate]


def test_bulk_matches_oracle(engine, world):
    """Many certificates in one bulk call: verdicts equal the oracle's Certificate::verify batch step
    with the same seeded coefficients."""
    seeds, keys, com = world
    rng = random.Random(3)
    certs = []
    for r in range(40):
        h = make_header(seeds, keys, com, author_idx=r % 4, round_=r + 1)
        c = make_cert(seeds, keys, com, h, voters=tuple(rng.sample(range(4), 3)))
        if r % 5 == 2:     # corrupt one vote's S
            k, s = c.votes[1]
            c.votes[1] = (k, s[:40] + bytes([s[40] ^ 4]) + s[41:])
        certs.append(c)
    zseed = bytes(range(32))
    got = pm.verify_certificates(certs, com, engine, zseed=zseed, cert_base=100)
    for j, c in enumerate(certs):
        want = o.crypto_verify_batch(o.digest32(c.digest_preimage()), c.votes, zseed, 100 + j)
        assert (got[j] is None) == want, j
        assert (got[j] is None) == (j % 5 != 2)
    # native wire path: same verdicts and coefficient indexing from the bincode frames
    native = pm.verify_certificate_frames([pm.encode_primary_message(c) for c in certs], com, engine,
                                          zseed=zseed, cert_base=100)
    assert [type(e) if e else None for e in native] == [type(e) if e else None for e in got]


def test_native_frames_committee_scale(engine):
    """Native path at a 100-validator committee (C2 shape, 67-vote certificates): honest frames
    accepted, one corrupted vote signature rejected, against the oracle's batch verdict."""
    from narwhal_amd import _lib
    rng = random.Random(5)
    seeds = [bytes([i + 1]) * 32 for i in range(100)]
    keys, _ = engine.sign_many(seeds, [bytes(32)] * 100)
    com = pm.Committee({k: (1, [0]) for k in keys})
    assert com.quorum_threshold() == 67
    order = sorted(range(100), key=lambda i: keys[i])
    certs = []
    for r in range(24):
        a = order[r % 100]
        h = pm.Header(keys[a], r + 1, {rng.randbytes(32): 0}, [rng.randbytes(32) for _ in range(67)])
        h.id = o.digest32(h.digest_preimage())
        h.signature = o.sign(seeds[a], h.id)
        voters = rng.sample(range(100), 67)
        v = pm.Vote(h.id, h.round, h.author, keys[0])
        d = o.digest32(v.digest_preimage())
        _, sigs = engine.sign_many([seeds[i] for i in voters], [d] * 67)
        c = pm.Certificate(h, [(keys[i], s) for i, s in zip(voters, sigs)])
        if r % 6 == 5:
            k, s = c.votes[30]
            c.votes[30] = (k, s[:5] + bytes([s[5] ^ 1]) + s[6:])
        certs.append(c)
    zseed = bytes([7]) * 32
    native = pm.verify_certificate_frames([pm.encode_primary_message(c) for c in certs], com, engine,
                                          zseed=zseed, cert_base=0)
    for j, c in enumerate(certs):
        want = o.crypto_verify_batch(o.digest32(c.digest_preimage()), c.votes, zseed, j)
        assert (native[j] is None) == want == (j % 6 != 5), j
    assert _lib.DAG_OK == 0
