"""CPU: the native certificate ingestion (nw_cert_batch_decode, narwhal_amd/csrc/nw_primary.cpp) —
bincode PrimaryMessage frames (primary/src/primary.rs:33-38,236; messages.rs:13-21,105-111,168-172),
base64 PublicKey strings (crypto/src/lib.rs:68-112) and the host-side checks of Certificate::verify
(messages.rs:189-215, Header::verify :48-67) — against the Python mirror (narwhal_amd.primary), on
the reference fixtures, randomized certificates, truncations and malformed keys.  The decode half
needs no GPU; the GPU half (nw_cert_batch_verify) is tests/test_gpu_primary.py."""
import base64
import hashlib
import random
import struct

import pytest

from narwhal_amd import _lib
from narwhal_amd import primary as pm


def _committee(golden, stake=1):
    keys = [bytes.fromhex(k["pk"]) for k in golden["reference_fixtures"]["keys"]]
    return pm.Committee({k: (stake, [0]) for k in keys}), keys


def _fixture_cert(golden):
    hd = golden["primary_fixtures"]["header"]
    h = pm.Header(bytes.fromhex(hd["author"]), hd["round"], {}, [bytes.fromhex(p) for p in hd["parents"]],
                  bytes.fromhex(hd["id"]), bytes.fromhex(hd["signature"]))
    votes = [(bytes.fromhex(k), bytes.fromhex(s)) for k, s in golden["primary_fixtures"]["votes"]]
    return pm.Certificate(h, votes)


def _pk_wire(s: bytes) -> bytes:
    return struct.pack("<Q", len(s)) + s


def _raw_cert_frame(author_b64, round_, payload, parents, id_, sig, votes):
    """A Certificate frame written field by field (payload / parents in the given wire order, keys
    as the given base64 strings), so non-canonical encodings can be built."""
    out = [struct.pack("<I", 2), _pk_wire(author_b64), struct.pack("<QQ", round_, len(payload))]
    for d, w in payload:
        out.append(d + struct.pack("<I", w))
    out.append(struct.pack("<Q", len(parents)))
    out.extend(parents)
    out.append(id_ + sig + struct.pack("<Q", len(votes)))
    for k64, s in votes:
        out.append(_pk_wire(k64) + s)
    return b"".join(out)


def _python_expect(frame, com):
    """(status, header_error, quorum_error, cert) the Python mirror assigns to a frame."""
    try:
        msg = pm.decode_primary_message(frame)
    except pm.SerializationError:
        return _lib.DAG_SERIALIZATION, None, None, None
    if not isinstance(msg, pm.Certificate):
        return _lib.DAG_NOT_CERTIFICATE, None, None, None
    if msg.is_genesis(com):
        return _lib.DAG_OK, None, None, msg
    h = msg.header
    herr = _lib.DAG_OK
    if com.stake(h.author) <= 0:
        herr = _lib.DAG_UNKNOWN_AUTHORITY
    elif any(not com.has_worker(h.author, w) for w in h.payload.values()):
        herr = _lib.DAG_MALFORMED_HEADER
    qerr = _lib.DAG_OK
    try:
        msg._quorum(com)
    except pm.AuthorityReuse:
        qerr = _lib.DAG_AUTHORITY_REUSE
    except pm.UnknownAuthority:
        qerr = _lib.DAG_UNKNOWN_AUTHORITY
    except pm.CertificateRequiresQuorum:
        qerr = _lib.DAG_REQUIRES_QUORUM
    return _lib.DAG_PENDING, herr, qerr, msg


def _check_against_python(frames, com):
    batch = pm.decode_certificate_frames(frames, com)
    assert len(batch) == len(frames)
    for i, f in enumerate(frames):
        v = batch.view(i)
        status, herr, qerr, cert = _python_expect(f, com)
        assert v["status"] == status, i
        if status == _lib.DAG_PENDING:
            assert (v["header_error"], v["quorum_error"]) == (herr, qerr), i
        if cert is not None:
            h = cert.header
            assert v["round"] == h.round and v["author"] == h.author and v["header_id"] == h.id, i
            assert v["header_sig"] == h.signature, i
            assert v["cert_preimage"] == cert.digest_preimage(), i
            assert v["votes"] == cert.votes, i
            if status == _lib.DAG_PENDING:
                assert v["header_preimage"] == h.digest_preimage(), i
    batch.close()


def test_reference_fixture_frame(golden):
    com, keys = _committee(golden)
    cert = _fixture_cert(golden)
    frame = pm.encode_primary_message(cert)
    batch = pm.decode_certificate_frames([frame], com)
    v = batch.view(0)
    assert v["status"] == _lib.DAG_PENDING and v["header_error"] == _lib.DAG_OK and v["quorum_error"] == _lib.DAG_OK
    # the digests the GPU will compute from these preimages are the reference's fixture digests
    assert hashlib.sha512(v["header_preimage"]).digest()[:32] == cert.header.id
    want = bytes.fromhex(golden["primary_fixtures"]["certificate_digest"])
    assert hashlib.sha512(v["cert_preimage"]).digest()[:32] == want
    assert v["votes"] == cert.votes
    _check_against_python([frame, frame + b"\x00\x01"], com)   # trailing bytes allowed (bincode 1.3)


def test_randomized_certificates_match_python(golden):
    com, keys = _committee(golden)
    com = pm.Committee({k: (1 + i, [0, 2]) for i, k in enumerate(keys)})
    rng = random.Random(11)
    outsider = bytes([3]) * 32
    frames = []
    for t in range(300):
        author = rng.choice(keys + [outsider])
        round_ = rng.choice([0, 1, rng.getrandbits(64)])
        digests = [rng.randbytes(32) for _ in range(rng.randrange(0, 4))]
        payload = [(rng.choice(digests), rng.choice([0, 2, 5])) for _ in range(rng.randrange(0, 5))] if digests else []
        parents = [rng.randbytes(32) for _ in range(rng.randrange(0, 6))]
        parents += rng.sample(parents, min(len(parents), rng.randrange(0, 2)))   # duplicates
        rng.shuffle(parents)
        id_ = bytes(32) if rng.random() < 0.1 else rng.randbytes(32)
        nv = rng.randrange(0, 6)
        voters = [rng.choice(keys + [outsider]) for _ in range(nv)]
        votes = [(base64.b64encode(k), rng.randbytes(64)) for k in voters]
        frames.append(_raw_cert_frame(base64.b64encode(author), round_, payload, parents, id_, rng.randbytes(64), votes))
    # genesis certificates (Header::default with a committee author)
    frames += [pm.encode_primary_message(g) for g in pm.Certificate.genesis(com)]
    _check_against_python(frames, com)


def test_truncations_and_variants(golden):
    com, keys = _committee(golden)
    frame = pm.encode_primary_message(_fixture_cert(golden))
    frames = [frame[:k] for k in range(0, len(frame), 7)] + [frame[:-1]]
    h = _fixture_cert(golden).header
    frames.append(pm.encode_primary_message(h))                                     # Header
    frames.append(pm.encode_primary_message(pm.Vote(h.id, 1, h.author, keys[0])))  # Vote
    frames.append(struct.pack("<I", 3) + bytes(8) + _pk_wire(base64.b64encode(keys[0])))  # CertificatesRequest
    frames.append(struct.pack("<I", 4) + frame[4:])                                 # no such variant
    frames.append(struct.pack("<I", 2) + struct.pack("<Q", 1 << 62))                # absurd key length
    batch = pm.decode_certificate_frames(frames, com)
    st = [batch.view(i)["status"] for i in range(len(frames))]
    n_trunc = len(frames) - 5
    assert all(s == _lib.DAG_SERIALIZATION for s in st[:n_trunc])
    assert st[n_trunc:] == [_lib.DAG_NOT_CERTIFICATE] * 3 + [_lib.DAG_SERIALIZATION] * 2
    _check_against_python(frames[:n_trunc] + frames[n_trunc + 3:], com)


@pytest.mark.parametrize("variant", ["canonical", "unpadded", "bad_pad", "trailing_bits", "bad_char", "short",
                                     "long", "one_symbol_tail", "pad_in_middle", "partial_pad", "over_pad"])
def test_base64_public_keys(golden, variant):
    """base64 0.13 decode rules (crypto/src/lib.rs:73-79); native decoder == Python mirror.  No
    reference vectors exist for malformed keys: these verdicts are parity unpinned."""
    com, keys = _committee(golden)
    k = keys[1]
    enc = base64.b64encode(k)                      # 44 chars, one '='
    s = {"canonical": enc, "unpadded": enc[:-1], "bad_pad": enc + b"=",
         "trailing_bits": enc[:42] + bytes([enc[42] + 1]) + b"=", "bad_char": b"*" + enc[1:],
         "short": base64.b64encode(k[:31]), "long": base64.b64encode(k + b"\x01\x02\x03"),
         "one_symbol_tail": enc[:-1] + b"AA", "pad_in_middle": enc[:20] + b"=" + enc[21:],
         # 34 bytes = 46 symbols + "==": base64 0.13 accepts a quad completed by only one '='
         "partial_pad": base64.b64encode(k + b"\x07\x00")[:-1],
         # 35 bytes = 47 symbols + "=": a second '=' lands on quad position 0
         "over_pad": base64.b64encode(k + b"\x07\x00\x01") + b"="}[variant]
    cert = _fixture_cert(golden)
    votes = [(base64.b64encode(kk), sg) for kk, sg in cert.votes]
    votes[1] = (s, votes[1][1])
    h = cert.header
    frame = _raw_cert_frame(base64.b64encode(h.author), h.round, [], sorted(h.parents), h.id, h.signature, votes)
    _check_against_python([frame], com)
    v = pm.decode_certificate_frames([frame], com).view(0)
    ok = variant in ("canonical", "unpadded", "long", "partial_pad")
    assert (v["status"] == _lib.DAG_PENDING) == ok
    if ok:
        assert v["votes"][1][0] == k


def test_b64_decode_rules():
    """The restated base64 0.13 decode_suffix rules on short strings (Python mirror; the native
    decoder agrees through test_base64_public_keys).  Parity unpinned: the crate is not vendored."""
    from narwhal_amd.primary import _b64_decode
    cases = {b"": b"", b"AA": b"\x00", b"AA=": b"\x00", b"AA==": b"\x00", b"AAA": b"\x00\x00",
             b"AAA=": b"\x00\x00", b"AAAA": b"\x00" * 3, b"A": None, b"A=": None, b"A==": None,
             b"AAA==": None, b"AA===": None, b"=": None, b"AB": None, b"AAB": None, b"AA=A": None,
             b"AAAAA": None, b"QQ": b"A", b"QUI": b"AB", b"AA*A": None}
    for s, want in cases.items():
        assert _b64_decode(s) == want, s


def test_host_check_order(golden):
    """Header author / worker-id checks and the quorum rules, in the reference's order."""
    com, keys = _committee(golden)
    cert = _fixture_cert(golden)
    h = cert.header
    stranger = bytes([9]) * 32
    cases = [
        (pm.Certificate(h, cert.votes), _lib.DAG_OK, _lib.DAG_OK),
        (pm.Certificate(pm.Header(stranger, 1, {}, h.parents, h.id, h.signature), cert.votes),
         _lib.DAG_UNKNOWN_AUTHORITY, _lib.DAG_OK),
        (pm.Certificate(pm.Header(h.author, 1, {bytes([5]) * 32: 7}, h.parents, h.id, h.signature), cert.votes),
         _lib.DAG_MALFORMED_HEADER, _lib.DAG_OK),
        (pm.Certificate(h, cert.votes[:2]), _lib.DAG_OK, _lib.DAG_REQUIRES_QUORUM),
        (pm.Certificate(h, cert.votes[:2] + cert.votes[:1]), _lib.DAG_OK, _lib.DAG_AUTHORITY_REUSE),
        (pm.Certificate(h, cert.votes[:1] + [(stranger, bytes(64))] * 2), _lib.DAG_OK, _lib.DAG_UNKNOWN_AUTHORITY),
    ]
    frames = [pm.encode_primary_message(c) for c, _, _ in cases]
    batch = pm.decode_certificate_frames(frames, com)
    for i, (_, herr, qerr) in enumerate(cases):
        v = batch.view(i)
        assert (v["status"], v["header_error"], v["quorum_error"]) == (_lib.DAG_PENDING, herr, qerr), i
    _check_against_python(frames, com)
