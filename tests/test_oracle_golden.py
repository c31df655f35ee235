"""CPU: pin the oracle against the golden fixtures before it is trusted as the checker."""
import struct

import ed25519_oracle as o


def test_rfc8032_known_answers(golden):
    for v in golden["rfc8032"]:
        seed, msg = bytes.fromhex(v["seed"]), bytes.fromhex(v["msg"])
        assert o.public_from_seed(seed).hex() == v["pk"]
        assert o.sign(seed, msg).hex() == v["sig"]
        assert o.verify_strict(bytes.fromhex(v["pk"]), msg, bytes.fromhex(v["sig"]))


def test_reference_fixture_keys(golden):
    """keys() of crypto_tests.rs:26-29 (ChaCha20 zero seed); SURVEY.md §4 lists the prefixes."""
    ks = golden["reference_fixtures"]["keys"]
    seeds = o.reference_fixture_seeds(4)
    assert seeds[0].hex().startswith("76b8e0ad") and seeds[0].hex().endswith("8b770dc7")
    prefixes = ["20fdbac9", "75e4174d", "631c1541", "beada061"]
    for s, k, pre in zip(seeds, ks, prefixes):
        assert s.hex() == k["seed"]
        assert o.public_from_seed(s).hex() == k["pk"]
        assert k["pk"].startswith(pre)
    assert golden["reference_fixtures"]["hello_digest"].startswith("c1527cd8")


def test_crypto_tests_verdicts(golden):
    """crypto_tests.rs:49-115 restated on the oracle."""
    rf = golden["reference_fixtures"]
    for name in ("verify_valid_signature", "verify_invalid_signature"):
        c = rf[name]
        assert o.verify_strict(bytes.fromhex(c["pk"]), bytes.fromhex(c["digest"]), bytes.fromhex(c["sig"])) == c["ok"]
    for name in ("verify_valid_batch", "verify_invalid_batch"):
        c = rf[name]
        votes = [(bytes.fromhex(k), bytes.fromhex(s)) for k, s in c["votes"]]
        for zb in (0, 1, 99):
            assert o.crypto_verify_batch(bytes.fromhex(c["digest"]), votes, bytes(32), zb) == c["ok"]


def test_primary_fixtures(golden):
    pf = golden["primary_fixtures"]
    hd = pf["header"]
    hid = o.header_digest(bytes.fromhex(hd["author"]), hd["round"], [], [bytes.fromhex(p) for p in hd["parents"]])
    assert hid.hex() == hd["id"]
    assert o.verify_strict(bytes.fromhex(hd["author"]), hid, bytes.fromhex(hd["signature"]))
    vd = o.vote_digest(hid, 1, bytes.fromhex(hd["author"]))
    assert vd.hex() == pf["vote_digest"]
    votes = [(bytes.fromhex(k), bytes.fromhex(s)) for k, s in pf["votes"]]
    assert all(o.verify_strict(k, vd, s) for k, s in votes)
    assert o.crypto_verify_batch(vd, votes, bytes(32))


def test_worker_batch_digest(golden):
    wb = golden["worker_batch"]
    ser = o.bincode_worker_batch([bytes(100), bytes(100)])
    assert ser.hex() == wb["serialized"] and len(ser) == 228 == wb["len"]
    assert o.digest32(ser).hex() == wb["digest"]
    assert wb["digest"].startswith("24d00f74") and wb["digest"].endswith("cd7331d8")


def test_sha512_vectors(golden):
    for v in golden["sha512"]:
        assert o.sha512(bytes.fromhex(v["msg"])).hex() == v["sha512"]


def test_chacha20_rfc8439(golden):
    c = golden["chacha20_rfc8439"]
    blk = o.chacha20_block(bytes.fromhex(c["key"]), c["counter"], bytes.fromhex(c["nonce"]))
    assert blk.hex() == c["block"]
    for v in golden["nwz_v1"]:
        zs = o.batch_coefficients(bytes.fromhex(v["zseed"]), v["batch_index"], len(v["z"]))
        assert [str(z) for z in zs] == v["z"]


def test_adversarial_strict_oracle(golden):
    for c in golden["adversarial_strict"]:
        got = o.verify_strict(bytes.fromhex(c["pk"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"]))
        assert got == c["strict"], c["name"]


def test_adversarial_batch_oracle_all(golden):
    """Re-derive every golden batch verdict on the oracle (196 batches, ~5 s), including the
    computed ``cancelling_pair_other_z`` cases."""
    names = {c["name"] for c in golden["adversarial_batch"]}
    assert "cancelling_pair_other_z" in names and "cancelling_pair" in names
    for c in golden["adversarial_batch"]:
        items = [(bytes.fromhex(k), bytes.fromhex(s), bytes.fromhex(m)) for k, s, m in c["items"]]
        pre = all(s[63] & 0xE0 == 0 and o.decompress(k) is not None for k, s, _ in items)
        zs = o.batch_coefficients(bytes.fromhex(c["zseed"]), c["batch_index"], len(items))
        got = pre and o.verify_batch_z([m for *_, m in items], [s for _, s, _ in items], [k for k, _, _ in items], zs)
        assert got == c["ok"], (c["name"], c["batch_index"])


def test_torsion_semantics_known_cases():
    """Spot-check the cofactorless batch vs strict split on hand-built cases."""
    T = o.small_order_generator()
    msg = bytes(32)
    a, r = 12345, 67890
    A = o.pt_mul(a, o.B_POINT)
    Ab = o.pt_compress(A)
    # (ii) R = identity, S = k a: strict rejects (R small order), batch accepts for every z
    Rb = o.pt_compress(o.IDENTITY)
    k = o.scalar_from_hash(o.sha512(Rb + Ab + msg))
    sig = Rb + (k * a % o.L).to_bytes(32, "little")
    assert not o.verify_strict(Ab, msg, sig)
    for z in (1, 2, 3, 2**127 + 1):
        assert o.verify_batch_z([msg], [sig], [Ab], [z])
    # (iii) R = rB + T8: batch accepts iff 8 | z
    Rp = o.pt_add(o.pt_mul(r, o.B_POINT), T)
    Rb = o.pt_compress(Rp)
    k = o.scalar_from_hash(o.sha512(Rb + Ab + msg))
    sig = Rb + ((r + k * a) % o.L).to_bytes(32, "little")
    assert not o.verify_strict(Ab, msg, sig)
    assert o.verify_batch_z([msg], [sig], [Ab], [8])
    assert not o.verify_batch_z([msg], [sig], [Ab], [4])
    assert struct.pack("<I", 1)   # keep struct import used
