"""GPU: Core-side batching (narwhal_amd.core) — a mixed batch of headers,
votes and certificates checked in a fixed number of GPU submissions gives exactly the verdicts of
the serial Core::sanitize_* loop (primary/src/core.rs:306-346) run message by message, and the
aggregators hand the same certificates and parents on."""
import random

import pytest

import ed25519_oracle as o
from narwhal_amd import core
from narwhal_amd import primary as pm

pytestmark = pytest.mark.gpu


def _header(seeds, keys, author, round_, parents=()):
    h = pm.Header(keys[author], round_, {}, parents)
    h.id = o.digest32(h.digest_preimage())
    h.signature = o.sign(seeds[author], h.id)
    return h


def _vote(seeds, keys, h, voter):
    v = pm.Vote(h.id, h.round, h.author, keys[voter])
    v.signature = o.sign(seeds[voter], o.digest32(v.digest_preimage()))
    return v


def _cert(seeds, keys, h, voters):
    d = o.digest32(pm.Vote(h.id, h.round, h.author, keys[0]).digest_preimage())
    return pm.Certificate(h, [(keys[i], o.sign(seeds[i], d)) for i in voters])


def _serial(msg, com, gc_round, current, engine, zseed, cert_index):
    """One message through the one-message verify forms, in the reference's order."""
    try:
        if isinstance(msg, pm.Header):
            if gc_round > msg.round:
                return core.TooOld
            msg.verify(com, engine)
        elif isinstance(msg, pm.Vote):
            if current.round > msg.round:
                return core.TooOld
            if not (msg.id == current.id and msg.origin == current.author and msg.round == current.round):
                return core.UnexpectedVote
            msg.verify(com, engine)
        else:
            if gc_round > msg.round():
                return core.TooOld
            # honest / corrupted votes: the verdict does not depend on the batch coefficients
            errs = pm.verify_certificates([msg], com, engine, zseed, cert_index)
            if errs[0] is not None:
                raise errs[0]
    except pm.DagError as e:
        return type(e)
    return None


def test_mixed_batch_matches_serial(engine):
    seeds = o.reference_fixture_seeds(7)
    keys = [o.public_from_seed(s) for s in seeds]
    com = pm.Committee({k: (1, [0]) for k in keys})        # quorum 5 of 7
    rng = random.Random(11)
    own = _header(seeds, keys, 0, 8)
    msgs = []
    for j in range(60):
        kind = j % 3
        r = rng.choice([3, 8, 9])
        if kind == 0:
            h = _header(seeds, keys, rng.randrange(7), r)
            if rng.random() < 0.2:
                h.signature = o.sign(seeds[(keys.index(h.author) + 1) % 7], h.id)
            msgs.append(h)
        elif kind == 1:
            v = _vote(seeds, keys, own if rng.random() < 0.7 else _header(seeds, keys, 1, 8), rng.randrange(7))
            if rng.random() < 0.2:
                v.signature = v.signature[:10] + bytes([v.signature[10] ^ 1]) + v.signature[11:]
            msgs.append(v)
        else:
            h = _header(seeds, keys, rng.randrange(7), r)
            c = _cert(seeds, keys, h, rng.sample(range(7), rng.choice([4, 5, 6])))
            if rng.random() < 0.2 and len(c.votes) >= 5:
                k, s = c.votes[2]
                c.votes[2] = (k, s[:40] + bytes([s[40] ^ 2]) + s[41:])
            msgs.append(c)
    zseed = bytes(range(32))
    got = core.sanitize_messages(msgs, com, gc_round=5, current_header=own, engine=engine, zseed=zseed)
    idx, want = 0, []
    for m in msgs:
        want.append(_serial(m, com, 5, own, engine, zseed, idx))
        idx += isinstance(m, pm.Certificate)
    assert [type(e) if e else None for e in got] == want
    kinds = set(want)
    assert {None, pm.InvalidSignature, core.TooOld, core.UnexpectedVote, pm.CertificateRequiresQuorum} <= kinds


def test_batcher_assembles_and_hands_parents(engine):
    seeds = o.reference_fixture_seeds(4)
    keys = [o.public_from_seed(s) for s in seeds]
    com = pm.Committee({k: (1, [0]) for k in keys})
    b = core.CoreBatcher(com, engine=engine)
    own = _header(seeds, keys, 0, 2)
    b.set_current_header(own)
    others = [_cert(seeds, keys, _header(seeds, keys, a, 2), (0, 1, 2)) for a in (1, 2)]
    msgs = [_vote(seeds, keys, own, i) for i in (1, 2, 3)] + others
    errs, assembled, parents = b.submit(msgs, zseed=bytes(32))
    assert errs == [None] * 5
    assert len(assembled) == 1 and assembled[0].header.id == own.id
    # own certificate (assembled from votes) + 2 received = quorum 3 for round 2
    assert len(parents) == 1 and parents[0][1] == 2
    assert [c.origin() for c in parents[0][0]] == [keys[0], keys[1], keys[2]]
    # the assembled certificate verifies as a received one would
    assembled[0].verify(com, engine)
