"""GPU parity: libnwcrypto (gfx950 HIP) vs the oracle and the golden fixtures.

The first block ports the reference's own tests (crypto/src/tests/crypto_tests.rs) onto the
drop-in API; the rest compares every golden vector, then checks size-independent properties at
the BASELINE.json C2 size (14,926 certificates x 67 votes).
"""
import asyncio
import os
import random

import numpy as np
import pytest

import ed25519_oracle as o

pytestmark = pytest.mark.gpu


def fx_keys():
    from narwhal_amd.crypto import PublicKey, SecretKey
    seeds = o.reference_fixture_seeds(4)
    out = []
    for s in seeds:
        pk = o.public_from_seed(s)
        out.append((PublicKey(pk), SecretKey(s + pk)))
    return out


# ----------------------------------------------------------------------------- crypto_tests.rs port
def test_import_export_public_key():
    from narwhal_amd.crypto import PublicKey
    public_key, _ = fx_keys().pop()
    export = public_key.encode_base64()
    assert PublicKey.decode_base64(export) == public_key


def test_import_export_secret_key():
    from narwhal_amd.crypto import SecretKey
    _, secret_key = fx_keys().pop()
    assert SecretKey.decode_base64(secret_key.encode_base64()) == secret_key


def test_generate_keypair_matches_reference_keys(golden):
    from narwhal_amd.crypto import generate_keypair
    stream = o.chacha20_stream(bytes(32), 128)
    pos = [0]

    def fill(n):
        b = stream[pos[0]:pos[0] + n]
        pos[0] += n
        return b

    for k in golden["reference_fixtures"]["keys"]:
        pk, sk = generate_keypair(fill)
        assert bytes(pk).hex() == k["pk"]
        assert sk.seed.hex() == k["seed"]


def test_verify_valid_signature():
    from narwhal_amd.crypto import Signature, digest_of
    public_key, secret_key = fx_keys().pop()
    digest = digest_of(b"Hello, world!")
    signature = Signature.new(digest, secret_key)
    assert signature.verify(digest, public_key) is None


def test_verify_invalid_signature():
    from narwhal_amd.crypto import CryptoError, Signature, digest_of
    public_key, secret_key = fx_keys().pop()
    signature = Signature.new(digest_of(b"Hello, world!"), secret_key)
    with pytest.raises(CryptoError):
        signature.verify(digest_of(b"Bad message!"), public_key)


def test_verify_valid_batch():
    from narwhal_amd.crypto import Signature, digest_of
    digest = digest_of(b"Hello, world!")
    keys = fx_keys()
    signatures = []
    for _ in range(3):
        pk, sk = keys.pop()
        signatures.append((pk, Signature.new(digest, sk)))
    assert Signature.verify_batch(digest, signatures) is None


def test_verify_invalid_batch():
    from narwhal_amd.crypto import CryptoError, Signature, digest_of
    digest = digest_of(b"Hello, world!")
    keys = fx_keys()
    signatures = []
    for _ in range(2):
        pk, sk = keys.pop()
        signatures.append((pk, Signature.new(digest, sk)))
    pk, _ = keys.pop()
    signatures.append((pk, Signature.default()))
    with pytest.raises(CryptoError):
        Signature.verify_batch(digest, signatures)


def test_signature_service():
    from narwhal_amd.crypto import SignatureService, digest_of
    public_key, secret_key = fx_keys().pop()
    service = SignatureService(secret_key)
    digest = digest_of(b"Hello, world!")
    signature = asyncio.run(service.request_signature(digest))
    assert signature.verify(digest, public_key) is None


# ----------------------------------------------------------------------------- golden vectors
def test_reference_fixture_signatures(engine, golden):
    rf = golden["reference_fixtures"]
    c = rf["verify_valid_signature"]
    seed = bytes.fromhex(rf["keys"][3]["seed"])
    pks, sigs = engine.sign_many([seed], [bytes.fromhex(c["digest"])])
    assert pks[0].hex() == c["pk"] and sigs[0].hex() == c["sig"]
    for name in ("verify_valid_signature", "verify_invalid_signature"):
        c = rf[name]
        assert engine.verify_strict(bytes.fromhex(c["digest"]), bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"])) == c["ok"]
    for name in ("verify_valid_batch", "verify_invalid_batch"):
        c = rf[name]
        d = bytes.fromhex(c["digest"])
        pks = [bytes.fromhex(k) for k, _ in c["votes"]]
        sigs = [bytes.fromhex(s) for _, s in c["votes"]]
        assert engine.verify_batch([d] * len(pks), pks, sigs, bytes(32), 0) == c["ok"]


def test_rfc8032(engine, golden):
    for v in golden["rfc8032"]:
        msg = bytes.fromhex(v["msg"])
        assert engine.verify_strict(msg, bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
        assert not engine.verify_strict(msg + b"x", bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))


def test_sha512_golden(engine, golden):
    msgs = [bytes.fromhex(v["msg"]) for v in golden["sha512"]]
    got = engine.sha512_many(msgs)
    assert [g.hex() for g in got] == [v["sha512"] for v in golden["sha512"]]
    assert engine.sha512(b"").hex() == o.sha512(b"").hex()
    wb = golden["worker_batch"]
    assert engine.sha512(bytes.fromhex(wb["serialized"]))[:32].hex() == wb["digest"]


def test_primary_fixtures(engine, golden):
    pf = golden["primary_fixtures"]
    hd = pf["header"]
    author = bytes.fromhex(hd["author"])
    assert engine.verify_strict(bytes.fromhex(hd["id"]), author, bytes.fromhex(hd["signature"]))
    vd = bytes.fromhex(pf["vote_digest"])
    pks = [bytes.fromhex(k) for k, _ in pf["votes"]]
    sigs = [bytes.fromhex(s) for _, s in pf["votes"]]
    assert engine.verify_strict_many([vd] * 4, pks, sigs) == [True] * 4
    assert engine.verify_batch([vd] * 4, pks, sigs, os.urandom(32), 0)


def test_adversarial_strict(engine, golden):
    cases = golden["adversarial_strict"]
    got = engine.verify_strict_many([bytes.fromhex(c["msg"]) for c in cases], [bytes.fromhex(c["pk"]) for c in cases],
                                    [bytes.fromhex(c["sig"]) for c in cases])
    bad = [c["name"] for c, g in zip(cases, got) if g != c["strict"]]
    assert not bad, bad


def test_adversarial_batch(engine, golden):
    bad = []
    for c in golden["adversarial_batch"]:
        items = [(bytes.fromhex(k), bytes.fromhex(s), bytes.fromhex(m)) for k, s, m in c["items"]]
        got = engine.verify_batch([m for *_, m in items], [k for k, _, _ in items], [s for _, s, _ in items],
                                  bytes.fromhex(c["zseed"]), c["batch_index"])
        if got != c["ok"]:
            bad.append((c["name"], c["batch_index"]))
    assert not bad, bad


def test_empty_and_mismatched(engine):
    assert engine.verify_batch([], [], [], bytes(32), 0)
    assert not engine.verify_batch([b"x"], [], [], bytes(32), 0)
    from narwhal_amd.crypto import Signature, Digest
    assert Signature.verify_batch(Digest(bytes(32)), []) is None


def test_generic_message_lengths(engine):
    """Worker-style 8-byte messages (worker/src/processor.rs:47) and other lengths through the
    generic hram path, vs the oracle."""
    rng = random.Random(5)
    for ln in (0, 8, 31, 32, 33, 47, 48, 100, 200):
        seed = bytes(rng.randrange(256) for _ in range(32))
        msg = bytes(rng.randrange(256) for _ in range(ln))
        sig = o.sign(seed, msg)
        pk = o.public_from_seed(seed)
        assert engine.verify_strict(msg, pk, sig), ln
        assert not engine.verify_strict(msg + b"\0", pk, sig), ln
    seeds = [bytes([i]) * 32 for i in range(1, 40)]
    msgs = [struct_le(i) for i in range(39)]
    pks, sigs = engine.sign_many(seeds, msgs)
    for i in range(39):
        assert sigs[i] == o.sign(seeds[i], msgs[i])
    assert engine.verify_batch(msgs, pks, sigs, bytes(32), 7)
    sigs[5] = sigs[5][:40] + bytes([sigs[5][40] ^ 1]) + sigs[5][41:]
    assert not engine.verify_batch(msgs, pks, sigs, bytes(32), 7)


def struct_le(i):
    return int(i).to_bytes(8, "little")


# ----------------------------------------------------------------------------- certificates
def test_certs_small_vs_oracle(engine):
    rng = random.Random(11)
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(7)]
    pks = [o.public_from_seed(s) for s in seeds]
    slots = engine.committee_load(pks, list(range(1, 8)))
    certs, sigs, signer, msgs = [], [], [], []
    for c in range(6):
        msg = bytes(rng.randrange(256) for _ in range(32))
        first = len(sigs)
        nv = [5, 0, 7, 3, 5, 1][c]
        for v in range(nv):
            k = (c + v) % 7
            s = o.sign(seeds[k], msg)
            if (c, v) in ((2, 3), (4, 0)):
                s = s[:33] + bytes([s[33] ^ 0x40]) + s[34:]     # corrupt S
            sigs.append(s)
            signer.append(slots[k])
        certs.append((first, nv))
        msgs.append(msg)
    cert_ok, sig_ok, stake = engine.verify_certs(certs, b"".join(sigs), signer, b"".join(msgs), bytes(32))
    for c, (first, nv) in enumerate(certs):
        votes = [(pks[(c + v) % 7], sigs[first + v]) for v in range(nv)]
        assert cert_ok[c] == o.crypto_verify_batch(msgs[c], votes, bytes(32), c), c
        exp = [o.verify_strict(pks[(c + v) % 7], msgs[c], sigs[first + v]) for v in range(nv)]
        assert sig_ok[first:first + nv] == exp
        assert stake[c] == sum(((c + v) % 7 + 1) for v in range(nv) if exp[v])


@pytest.fixture(scope="module")
def c2(engine):
    from narwhal_amd import workload
    com = workload.make_committee(100, engine)
    slots = engine.committee_load_np(com.pks, com.stake)
    certs = workload.make_certificates(com, 14926, 67, engine)
    return com, slots, certs


def test_c2_all_valid(engine, c2):
    """BASELINE C2 size: 14,926 certificates x 67 votes = 1,000,042 signatures."""
    com, slots, cs = c2
    assert cs.nsigs == 1000042
    cert_ok, sig_ok, stake = engine.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs,
                                                    os.urandom(32))
    assert cert_ok.all() and sig_ok.all()
    assert (stake == 67).all()
    assert stake[0] >= com.quorum_threshold()


def test_c2_corruptions_localized(engine, c2):
    """Property at full size: exactly the certificates holding a corrupted vote fail, and the
    per-signature bitmap flags exactly the corrupted votes."""
    com, slots, cs = c2
    rng = np.random.default_rng(3)
    sigs = cs.sigs.copy()
    bad = rng.choice(cs.nsigs, 300, replace=False)
    kind = rng.integers(0, 3, size=bad.shape[0])
    for b, k in zip(bad, kind):
        if k == 0:
            sigs[b, 40] ^= 1            # S corrupted
        elif k == 1:
            sigs[b, 3] ^= 0x10          # R corrupted
        else:
            sigs[b, 63] |= 0xE0         # S high bits
    cert_ok, sig_ok, _ = engine.verify_certs_np(cs.cert_first, cs.cert_n, sigs, slots[cs.signer], cs.msgs,
                                                os.urandom(32))
    exp_sig = np.ones(cs.nsigs, bool)
    exp_sig[bad] = False
    assert (sig_ok.astype(bool) == exp_sig).all()
    bad_certs = set((bad // 67).tolist())
    exp_cert = np.array([c not in bad_certs for c in range(cs.ncerts)])
    assert (cert_ok.astype(bool) == exp_cert).all()
    # spot-check two failing and one passing certificate against the oracle's batch equation
    for c in list(bad_certs)[:2] + [next(c for c in range(cs.ncerts) if c not in bad_certs)]:
        f, n = int(cs.cert_first[c]), int(cs.cert_n[c])
        votes = [(bytes(com.pks[cs.signer[f + v]]), bytes(sigs[f + v])) for v in range(n)]
        assert o.crypto_verify_batch(bytes(cs.msgs[c]), votes, bytes(32), c) == bool(cert_ok[c])


# ----------------------------------------------------------------------------- worker load (A13)
def test_verify_batches_worker_chunks(engine):
    """worker/src/processor.rs:75-79: fixed keypairs, 8-byte LE messages i, the batch split into
    64 chunks [count*c/64, min(count, count*(c+1)/64)), one dalek::verify_batch per chunk — here one
    nw_verify_batches call.  Some chunks carry a bad signature (wrong message / bit flip / S >= l);
    every chunk verdict and per-signature verdict is checked against the oracle."""
    rng = random.Random(21)
    count = 300
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(count)]
    msgs = [struct_le(i) for i in range(count)]
    pks, sigs = engine.sign_many(seeds, msgs)
    slots = engine.committee_load(pks)
    bad = {7: "flip", 100: "msg", 201: "s_ge_l"}
    for i, how in bad.items():
        s = bytearray(sigs[i])
        if how == "flip":
            s[3] ^= 0x10
        elif how == "msg":
            s = bytearray(o.sign(seeds[i], b"other"))
        else:
            sv = int.from_bytes(s[32:], "little") + o.L
            s[32:] = sv.to_bytes(32, "little")
        sigs[i] = bytes(s)
    chunks = [((count * c) // 64, min(count, (count * (c + 1)) // 64) - (count * c) // 64) for c in range(64)]
    zseed = bytes(rng.randrange(256) for _ in range(32))
    batch_ok, sig_ok = engine.verify_batches(chunks, msgs, slots, sigs, zseed, 1000)
    for c, (f, n) in enumerate(chunks):
        zs = o.batch_coefficients(zseed, 1000 + c, n)
        want = o.verify_batch_z(msgs[f:f + n], sigs[f:f + n], pks[f:f + n], zs)
        assert batch_ok[c] == want, c
        assert want == all(i not in bad for i in range(f, f + n))
    assert sig_ok == [o.verify_strict(pks[i], msgs[i], sigs[i]) for i in range(count)]
