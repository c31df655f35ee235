"""CPU: host logic of narwhal_amd.primary (the Certificate/Header/Vote callers): the reference's
bincode wire format (PrimaryMessage, primary/src/primary.rs:33-38; PublicKey as base64 string,
crypto/src/lib.rs:94-112), digest pre-images (primary/src/messages.rs:70-84,145-153,226-234) against
the golden fixtures, and the quorum / genesis rules (:189-215).  No GPU: digests and signature checks
are exercised by tests/test_gpu_primary.py."""
import hashlib
import struct

import pytest

from narwhal_amd import primary as pm


def _committee(golden, stake=1):
    keys = [bytes.fromhex(k["pk"]) for k in golden["reference_fixtures"]["keys"]]
    return pm.Committee({k: (stake, [0]) for k in keys}), keys


def _fixture_header(golden):
    hd = golden["primary_fixtures"]["header"]
    return pm.Header(bytes.fromhex(hd["author"]), hd["round"], {}, [bytes.fromhex(p) for p in hd["parents"]],
                     bytes.fromhex(hd["id"]), bytes.fromhex(hd["signature"]))


def test_digest_preimages_match_golden(golden):
    h = _fixture_header(golden)
    assert hashlib.sha512(h.digest_preimage()).digest()[:32] == h.id
    c = pm.Certificate(h, [])
    want = bytes.fromhex(golden["primary_fixtures"]["certificate_digest"])
    assert hashlib.sha512(c.digest_preimage()).digest()[:32] == want
    v = pm.Vote(h.id, h.round, h.author, h.author)
    assert hashlib.sha512(v.digest_preimage()).digest()[:32] == bytes.fromhex(golden["primary_fixtures"]["vote_digest"])


def test_genesis_parents_are_genesis_certificate_digests(golden):
    com, keys = _committee(golden)
    parents = sorted(hashlib.sha512(c.digest_preimage()).digest()[:32] for c in pm.Certificate.genesis(com))
    assert parents == sorted(bytes.fromhex(p) for p in golden["primary_fixtures"]["header"]["parents"])


def test_wire_roundtrip(golden):
    h = _fixture_header(golden)
    h.payload = {bytes([7]) * 32: 0, bytes([1]) * 32: 3}
    votes = [(bytes.fromhex(k), bytes.fromhex(s)) for k, s in golden["primary_fixtures"]["votes"]]
    for msg in (h, pm.Vote(h.id, 1, h.author, votes[0][0], votes[0][1]), pm.Certificate(h, votes)):
        buf = pm.encode_primary_message(msg)
        back = pm.decode_primary_message(buf)
        assert type(back) is type(msg) and pm.encode_primary_message(back) == buf
    cert = pm.Certificate(h, votes)
    buf = pm.encode_primary_message(cert)
    # 116 B per vote on the wire: u64 len + 44-char base64 key + 64-B signature
    assert len(pm.encode_primary_message(pm.Certificate(h, votes + votes[:1]))) - len(buf) == 116
    assert struct.unpack("<I", buf[:4])[0] == 2
    with pytest.raises(pm.SerializationError):
        pm.decode_primary_message(buf[:-1])
    # bincode::deserialize (bincode 1.3) allows trailing bytes
    assert pm.encode_primary_message(pm.decode_primary_message(buf + b"\0")) == buf


def test_quorum_rules(golden):
    com, keys = _committee(golden)
    assert com.quorum_threshold() == 3 and com.validity_threshold() == 2
    h = _fixture_header(golden)
    sig = bytes(64)
    pm.Certificate(h, [(k, sig) for k in keys[:3]])._quorum(com)
    with pytest.raises(pm.CertificateRequiresQuorum):
        pm.Certificate(h, [(k, sig) for k in keys[:2]])._quorum(com)
    with pytest.raises(pm.AuthorityReuse):
        pm.Certificate(h, [(keys[0], sig), (keys[1], sig), (keys[0], sig)])._quorum(com)
    with pytest.raises(pm.UnknownAuthority):
        pm.Certificate(h, [(keys[0], sig), (bytes(32), sig), (keys[1], sig)])._quorum(com)


def test_genesis_detection(golden):
    com, keys = _committee(golden)
    for g in pm.Certificate.genesis(com):
        assert g.is_genesis(com)
    assert not pm.Certificate(pm.Header(bytes(32), 0)).is_genesis(com)
    assert not pm.Certificate(pm.Header(keys[0], 1)).is_genesis(com)
