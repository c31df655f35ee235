"""CPU: the Core-side batching host logic (narwhal_amd.core) — the aggregators
(primary/src/aggregators.rs) and the arrival-order semantics of the batched sanitize
(primary/src/core.rs:306-346) — with an oracle-backed engine test double standing in for
libnwcrypto (test infrastructure: the product path only ever runs on the GPU engine)."""
import pytest

import ed25519_oracle as o
from narwhal_amd import core
from narwhal_amd import primary as pm


class OracleEngine:
    """Test double: the two engine calls sanitize_messages makes for headers and votes."""

    def __init__(self):
        self.calls = []

    def sha512_many(self, msgs):
        self.calls.append("sha512_many")
        return [o.sha512(m) for m in msgs]

    def verify_strict_many(self, msgs, pks, sigs):
        self.calls.append("verify_strict_many")
        return [o.verify_strict(k, m, s) for m, k, s in zip(msgs, pks, sigs)]


@pytest.fixture(scope="module")
def world():
    seeds = o.reference_fixture_seeds(4)
    keys = [o.public_from_seed(s) for s in seeds]
    com = pm.Committee({k: (1, [0]) for k in keys})
    return seeds, keys, com


def _header(seeds, keys, author, round_):
    h = pm.Header(keys[author], round_, {}, [])
    h.id = o.digest32(h.digest_preimage())
    h.signature = o.sign(seeds[author], h.id)
    return h


def _vote(seeds, keys, h, voter):
    v = pm.Vote(h.id, h.round, h.author, keys[voter])
    v.signature = o.sign(seeds[voter], o.digest32(v.digest_preimage()))
    return v


def test_votes_aggregator(world):
    seeds, keys, com = world
    h = _header(seeds, keys, 0, 1)
    agg = core.VotesAggregator()
    assert agg.append(_vote(seeds, keys, h, 0), com, h) is None
    assert agg.append(_vote(seeds, keys, h, 1), com, h) is None
    with pytest.raises(pm.AuthorityReuse):
        agg.append(_vote(seeds, keys, h, 1), com, h)
    cert = agg.append(_vote(seeds, keys, h, 2), com, h)      # quorum 3 of 4
    assert cert is not None and [k for k, _ in cert.votes] == keys[:3]
    assert agg.append(_vote(seeds, keys, h, 3), com, h) is None   # weight reset: quorum once


def test_certificates_aggregator(world):
    seeds, keys, com = world
    certs = [pm.Certificate(_header(seeds, keys, a, 2)) for a in range(4)]
    agg = core.CertificatesAggregator()
    assert agg.append(certs[0], com) is None
    assert agg.append(certs[0], com) is None                  # same origin: ignored
    assert agg.append(certs[1], com) is None
    assert agg.append(certs[2], com) == certs[:3]
    # weight is not reset (aggregators.rs:78): the next distinct origin re-triggers
    assert agg.append(certs[3], com) == [certs[3]]


def test_sanitize_batch_headers_votes(world):
    seeds, keys, com = world
    own = _header(seeds, keys, 0, 5)
    other = _header(seeds, keys, 1, 5)
    bad_sig = _header(seeds, keys, 2, 5)
    bad_sig.signature = o.sign(seeds[3], bad_sig.id)
    bad_id = _header(seeds, keys, 3, 5)
    bad_id.round = 6
    old = _header(seeds, keys, 1, 1)
    v_ok = _vote(seeds, keys, own, 1)
    v_bad = _vote(seeds, keys, own, 2)
    v_bad.signature = bytes(64)
    v_unexp = _vote(seeds, keys, other, 1)
    v_old = _vote(seeds, keys, _header(seeds, keys, 0, 4), 1)
    stranger = o.public_from_seed(bytes([7]) * 32)
    v_unknown = pm.Vote(own.id, own.round, own.author, stranger, bytes(64))
    msgs = [other, bad_sig, bad_id, old, v_ok, v_bad, v_unexp, v_old, v_unknown]
    want = [None, pm.InvalidSignature, pm.InvalidHeaderId, core.TooOld, None, pm.InvalidSignature,
            core.UnexpectedVote, core.TooOld, pm.UnknownAuthority]
    eng = OracleEngine()
    got = core.sanitize_messages(msgs, com, gc_round=2, current_header=own, engine=eng)
    assert [type(e) if e else None for e in got] == want
    assert eng.calls == ["sha512_many", "verify_strict_many"]     # one submission of each


def test_core_batcher_votes_to_certificate(world):
    seeds, keys, com = world
    own = _header(seeds, keys, 0, 3)
    b = core.CoreBatcher(com, engine=OracleEngine())
    b.set_current_header(own)
    dup = _vote(seeds, keys, own, 1)
    errs, assembled, parents = b.submit([_vote(seeds, keys, own, 0), dup, dup, _vote(seeds, keys, own, 2)])
    assert [type(e) if e else None for e in errs] == [None, None, pm.AuthorityReuse, None]
    assert len(assembled) == 1 and assembled[0].header is own
    assert [k for k, _ in assembled[0].votes] == [keys[0], keys[1], keys[2]]
    assert parents == []    # one certificate of round 3 is not a quorum of certificates
    b.advance_gc(60)
    assert b.gc_round == 10
    errs, _, _ = b.submit([_header(seeds, keys, 1, 9)])
    assert isinstance(errs[0], core.TooOld)
