"""CPU: the C restatement of dalek (oracle/nw_ref.c, the timed CPU baseline) agrees with the
Python oracle and the golden vectors — Straus (n < 190 points) and Pippenger (n >= 190) paths."""
import os
import random

import pytest

import ed25519_oracle as o

nw_ref = pytest.importorskip("nw_ref", reason="oracle/libnwref.so not built")


def test_sha512(golden):
    for v in golden["sha512"]:
        assert nw_ref.sha512(bytes.fromhex(v["msg"])).hex() == v["sha512"]


def test_decompress_matches_oracle():
    rng = random.Random(3)
    encs = [bytes(32), (o.P + 1).to_bytes(32, "little"), ((1 << 255) | 1).to_bytes(32, "little")]
    encs += [bytes(rng.randrange(256) for _ in range(32)) for _ in range(200)]
    for e in encs:
        ref = o.decompress(e)
        got = nw_ref.decompress(e)
        assert (got is None) == (ref is None)
        if ref is not None:
            assert got == o.pt_compress(ref)


def test_strict_golden(golden):
    for c in golden["adversarial_strict"] + [dict(name="rfc", pk=v["pk"], msg=v["msg"], sig=v["sig"], strict=True)
                                             for v in golden["rfc8032"]]:
        got = nw_ref.verify_strict(bytes.fromhex(c["pk"]), bytes.fromhex(c["msg"]), bytes.fromhex(c["sig"]))
        assert got == c["strict"], c["name"]


def test_batch_golden(golden):
    for c in golden["adversarial_batch"]:
        items = [(bytes.fromhex(k), bytes.fromhex(s), bytes.fromhex(m)) for k, s, m in c["items"]]
        if len({m for *_, m in items}) != 1:
            continue
        got = nw_ref.crypto_verify_batch(items[0][2], [(k, s) for k, s, _ in items], bytes.fromhex(c["zseed"]),
                                         c["batch_index"])
        assert got == c["ok"], c["name"]


@pytest.mark.parametrize("n", [1, 3, 94, 95, 120])
def test_straus_and_pippenger_sizes(n):
    """2n+1 points: n = 94 -> 189 (Straus), n = 95 -> 191 (Pippenger w=6)."""
    rng = random.Random(n)
    msg = bytes(rng.randrange(256) for _ in range(32))
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    votes = [(o.public_from_seed(s), o.sign(s, msg)) for s in seeds]
    assert nw_ref.crypto_verify_batch(msg, votes, bytes(32), 0)
    j = rng.randrange(n)
    bad = list(votes)
    bad[j] = (bad[j][0], bad[j][1][:40] + bytes([bad[j][1][40] ^ 4]) + bad[j][1][41:])
    assert not nw_ref.crypto_verify_batch(msg, bad, bytes(32), 0)


def test_torsion_batch_agrees_with_oracle():
    """Mixed-order R in a 100-vote batch (Pippenger): verdict depends on z exactly as the oracle says."""
    rng = random.Random(9)
    msg = bytes(32)
    T = o.small_order_generator()
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(99)]
    votes = [(o.public_from_seed(s), o.sign(s, msg)) for s in seeds]
    a, r = rng.randrange(1, o.L), rng.randrange(1, o.L)
    Ab = o.pt_compress(o.pt_mul(a, o.B_POINT))
    Rb = o.pt_compress(o.pt_add(o.pt_mul(r, o.B_POINT), o.pt_mul(4, T)))   # order-2 torsion
    k = o.scalar_from_hash(o.sha512(Rb + Ab + msg))
    votes.append((Ab, Rb + ((r + k * a) % o.L).to_bytes(32, "little")))
    for bidx in range(6):
        zs = o.batch_coefficients(bytes(32), bidx, len(votes))
        want = o.verify_batch_z([msg] * len(votes), [s for _, s in votes], [k for k, _ in votes], zs)
        assert nw_ref.crypto_verify_batch(msg, votes, bytes(32), bidx) == want == (zs[-1] % 2 == 0)


def test_verify_batch_msgs_matches_oracle():
    """Per-signature-message batches (worker/src/processor.rs:78) agree with the Python oracle."""
    import random
    rng = random.Random(9)
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(6)]
    msgs = [i.to_bytes(8, "little") for i in range(6)]
    pks = [o.public_from_seed(s) for s in seeds]
    sigs = [o.sign(s, m) for s, m in zip(seeds, msgs)]
    zseed = bytes(range(32))
    assert nw_ref.verify_batch_msgs(msgs, pks, sigs, zseed, 3)
    assert o.verify_batch_z(msgs, sigs, pks, o.batch_coefficients(zseed, 3, 6))
    bad = list(sigs)
    bad[2] = o.sign(seeds[2], b"x")
    assert not nw_ref.verify_batch_msgs(msgs, pks, bad, zseed, 3)
    assert not o.verify_batch_z(msgs, bad, pks, o.batch_coefficients(zseed, 3, 6))
