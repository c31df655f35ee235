"""GPU parity of both key paths against the golden vectors and the oracle.

* Cached keys (committee comb tables) at every key window the library can pick, including W20,
  the window bench.py's committee mode runs at C2.
* Uncached keys (the variable-base path: per-signature decompression + windowed scalar
  multiplication for strict verify; the Pippenger MSM for batch verify).  The reference verifies
  any key (crypto/src/lib.rs:202,216,218); the calls must leave the key cache unchanged.
* The split of one batch across shards: per-shard partial sums + an identity
  test of their sum.
"""
import random

import pytest

import ed25519_oracle as o

pytestmark = pytest.mark.gpu


def _strict_cases(golden):
    cases = golden["adversarial_strict"]
    return ([bytes.fromhex(c["msg"]) for c in cases], [bytes.fromhex(c["pk"]) for c in cases],
            [bytes.fromhex(c["sig"]) for c in cases], [c["strict"] for c in cases], [c["name"] for c in cases])


def _all_keys(golden):
    ks = {bytes.fromhex(c["pk"]) for c in golden["adversarial_strict"]}
    for c in golden["adversarial_batch"]:
        ks.update(bytes.fromhex(k) for k, _, _ in c["items"])
    return sorted(ks)


def _batch_mismatches(eng, golden):
    bad = []
    for c in golden["adversarial_batch"]:
        items = [(bytes.fromhex(k), bytes.fromhex(s), bytes.fromhex(m)) for k, s, m in c["items"]]
        got = eng.verify_batch([m for *_, m in items], [k for k, _, _ in items], [s for _, s, _ in items],
                               bytes.fromhex(c["zseed"]), c["batch_index"])
        if got != c["ok"]:
            bad.append((c["name"], c["batch_index"]))
    return bad


# ----------------------------------------------------------------------------- cached, every window
@pytest.mark.parametrize("window", [8, 9, 12, 13, 16, 20])
def test_cached_windows_full_golden(window, golden):
    """Every golden strict and batch verdict with all 60 golden keys in the committee cache."""
    from narwhal_amd import _lib
    eng = _lib.Engine(device=0, key_window=window)
    try:
        eng.committee_load(_all_keys(golden))
        assert eng.key_window() == window
        n0 = eng.committee_size()
        msgs, pks, sigs, want, names = _strict_cases(golden)
        got = eng.verify_strict_many(msgs, pks, sigs)
        assert [nm for nm, g, w in zip(names, got, want) if g != w] == []
        assert _batch_mismatches(eng, golden) == []
        assert eng.committee_size() == n0
    finally:
        eng.close()


# ----------------------------------------------------------------------------- uncached keys
@pytest.fixture(scope="module")
def bare():
    """An engine whose key cache stays empty."""
    from narwhal_amd import _lib
    eng = _lib.Engine(device=0, key_window=-1)
    yield eng
    eng.close()


def test_uncached_strict_golden(bare, golden):
    msgs, pks, sigs, want, names = _strict_cases(golden)
    got = bare.verify_strict_many(msgs, pks, sigs)
    assert [nm for nm, g, w in zip(names, got, want) if g != w] == []
    for v in golden["rfc8032"]:
        msg = bytes.fromhex(v["msg"])
        assert bare.verify_strict(msg, bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
        assert not bare.verify_strict(msg + b"x", bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]))
    assert bare.committee_size() == 0


@pytest.mark.parametrize("size", [1, 5, 16, 17])
def test_uncached_strict_golden_small_calls(bare, golden, size):
    """Calls of at most 4,096 signatures take the quad-split kernel (k_verify_var<true>: one quad
    per signature, 16 per one-wave block): every golden strict verdict in calls of `size`
    signatures (one block, a partial block, two blocks), ragged last call included."""
    msgs, pks, sigs, want, names = _strict_cases(golden)
    got = []
    for f in range(0, len(msgs), size):
        got += bare.verify_strict_many(msgs[f:f + size], pks[f:f + size], sigs[f:f + size])
    assert [nm for nm, g, w in zip(names, got, want) if g != w] == []
    assert any(want) and not all(want)


def test_uncached_strict_lane_kernel(bare, golden):
    """Above 4,096 signatures the lane-per-signature kernel (k_verify_var<false>): the golden strict
    cases after 4,100 fresh honest signatures, three of them corrupted, in one call."""
    rng = random.Random(4100)
    n = 4100
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    hm = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    hp, hs = bare.sign_many(seeds, hm)
    for i in (0, 2047, 4099):
        s = bytearray(hs[i])
        s[i % 32] ^= 0x10
        hs[i] = bytes(s)
    msgs, pks, sigs, want, names = _strict_cases(golden)
    got = bare.verify_strict_many(hm + msgs, hp + pks, hs + sigs)
    assert got[:n] == [i not in (0, 2047, 4099) for i in range(n)]
    assert [nm for nm, g, w in zip(names, got[n:], want) if g != w] == []


def test_uncached_batch_golden(bare, golden):
    """All 196 golden batches (every adversarial class, cancelling pairs) through the MSM."""
    assert _batch_mismatches(bare, golden) == []
    rf = golden["reference_fixtures"]
    for name in ("verify_valid_batch", "verify_invalid_batch"):
        c = rf[name]
        d = bytes.fromhex(c["digest"])
        pks = [bytes.fromhex(k) for k, _ in c["votes"]]
        sigs = [bytes.fromhex(s) for _, s in c["votes"]]
        assert bare.verify_batch([d] * len(pks), pks, sigs, bytes(32), 0) == c["ok"]
    assert bare.committee_size() == 0


def test_uncached_worker_chunks_vs_oracle(bare):
    """worker/src/processor.rs:75-79 without a key cache: 64 verify_batch chunks of fresh keys and
    8-byte messages in one nw_verify_batches_pk call; bad signatures in some chunks."""
    rng = random.Random(31)
    count = 1000
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(count)]
    msgs = [i.to_bytes(8, "little") for i in range(count)]
    pks, sigs = bare.sign_many(seeds, msgs)
    for i in (7, 300, 301, 999):
        s = bytearray(sigs[i])
        s[40] ^= 4
        sigs[i] = bytes(s)
    sigs[500] = sigs[500][:32] + (int.from_bytes(sigs[500][32:], "little") + o.L).to_bytes(32, "little")
    chunks = [min(count, (count * (c + 1)) // 64) - (count * c) // 64 for c in range(64)]
    zseed = bytes(rng.randrange(256) for _ in range(32))
    got = bare.verify_batches_pk(chunks, msgs, pks, sigs, zseed, 4000)
    f = 0
    for c, n in enumerate(chunks):
        zs = o.batch_coefficients(zseed, 4000 + c, n)
        want = o.verify_batch_z(msgs[f:f + n], sigs[f:f + n], pks[f:f + n], zs)
        assert got[c] == want, c
        assert want == all(i not in (7, 300, 301, 999, 500) for i in range(f, f + n))
        f += n
    assert bare.committee_size() == 0


@pytest.mark.parametrize("ml", [8, 32])
def test_uncached_fixed_length_messages_vs_oracle(bare, ml):
    """Messages of one length back to back in one buffer (numpy rows, as bench.py's msm leg and a
    Rust caller with a flat buffer): the upload sends the block alone and k_msm_prep addresses
    message i at i * len.  Verdicts equal the per-message upload's (separate bytes objects) and the
    oracle's, with bad signatures in some chunks."""
    import numpy as np
    rng = random.Random(41 + ml)
    count = 700
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(count)]
    msgs = [bytes(rng.randrange(256) for _ in range(ml)) for _ in range(count)]
    pks, sigs = bare.sign_many(seeds, msgs)
    bad = (3, 250, 251, 699)
    for i in bad:
        s = bytearray(sigs[i])
        s[41] ^= 2
        sigs[i] = bytes(s)
    chunks = [(count * (c + 1)) // 16 - (count * c) // 16 for c in range(16)]
    zseed = bytes(rng.randrange(256) for _ in range(32))
    listed = bare.verify_batches_pk(chunks, msgs, pks, sigs, zseed, 77)
    flat = np.frombuffer(b"".join(msgs), np.uint8).reshape(count, ml)
    call = bare.prepare_batches_pk_call(chunks, flat, np.frombuffer(b"".join(pks), np.uint8).reshape(count, 32),
                                        np.frombuffer(b"".join(sigs), np.uint8).reshape(count, 64))
    fixed = [bool(x) for x in call(zseed, 77)]
    firsts = [sum(chunks[:c]) for c in range(16)]
    want = [all(not (f <= i < f + n) for i in bad) for f, n in zip(firsts, chunks)]
    assert listed == want and fixed == want
    for c in (0, 5, 15):
        f, n = firsts[c], chunks[c]
        zs = o.batch_coefficients(zseed, 77 + c, n)
        assert o.verify_batch_z(msgs[f:f + n], sigs[f:f + n], pks[f:f + n], zs) == want[c]


@pytest.mark.parametrize("ragged", [False, True])
def test_uncached_large_call_vs_small_calls(bare, ragged):
    """One 20,000-signature nw_verify_batches_pk call (multi-chunk windows in every batch): the
    verdicts equal those of the same batches verified by 5,000-signature calls with matching batch
    indices (coefficients are keyed by the global batch index), and the oracle's on a bad and a
    good chunk.
    ragged: 8- and 32-byte messages interleaved at random (per-message staging, uneven slices)."""
    rng = random.Random(77 + ragged)
    count, nch = 20000, 16
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(count)]
    msgs = [i.to_bytes(8, "little") * (4 if ragged and rng.random() < 0.5 else 1) for i in range(count)]
    pks, sigs = [None] * count, [None] * count
    for ml in (8, 32):   # nw_sign_many signs equal-length messages
        ix = [i for i in range(count) if len(msgs[i]) == ml]
        if ix:
            p_, s_ = bare.sign_many([seeds[i] for i in ix], [msgs[i] for i in ix])
            for k, i in enumerate(ix):
                pks[i], sigs[i] = p_[k], s_[k]
    bad = (5, 4999, 5000, 15001, 19999)
    for i in bad:
        s = bytearray(sigs[i])
        s[40] ^= 4
        sigs[i] = bytes(s)
    chunks = [(count * (c + 1)) // nch - (count * c) // nch for c in range(nch)]
    zseed = bytes(rng.randrange(256) for _ in range(32))
    got = bare.verify_batches_pk(chunks, msgs, pks, sigs, zseed, 900)
    firsts = [sum(chunks[:c]) for c in range(nch)]
    want = [all(not (f <= i < f + n) for i in bad) for f, n in zip(firsts, chunks)]
    assert got == want
    small = []
    for g in range(0, nch, 4):   # 5,000 signatures per call: the unsliced path
        f0, f1 = firsts[g], firsts[g] + sum(chunks[g:g + 4])
        small += bare.verify_batches_pk(chunks[g:g + 4], msgs[f0:f1], pks[f0:f1], sigs[f0:f1], zseed, 900 + g)
    assert small == got
    for c in (3, 7):
        f, n = firsts[c], chunks[c]
        zs = o.batch_coefficients(zseed, 900 + c, n)
        assert o.verify_batch_z(msgs[f:f + n], sigs[f:f + n], pks[f:f + n], zs) == got[c]


@pytest.mark.parametrize("n", [1, 67, 700, 6667])
def test_uncached_batch_sizes(bare, n):
    """Both MSM window sizes (C = 7 below 512 signatures, 8 above) and multi-chunk windows
    (2n > 2,048 entries): honest batches accept; one flipped S bit, a swapped message or an R of
    small order (class ii, batch-accepted) behave as the oracle says."""
    rng = random.Random(n)
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    msg = bytes(rng.randrange(256) for _ in range(32))
    pks, sigs = bare.sign_many(seeds, [msg] * n)
    zseed = bytes(rng.randrange(256) for _ in range(32))
    assert bare.verify_batch([msg] * n, pks, sigs, zseed, 3)
    j = n // 2
    bad = list(sigs)
    bad[j] = bad[j][:40] + bytes([bad[j][40] ^ 1]) + bad[j][41:]
    assert not bare.verify_batch([msg] * n, pks, bad, zseed, 3)
    # class (ii): R = identity, S = k a  -> rejected by strict, accepted by the batch equation
    import adversarial_mix as am
    a, _ = am.secret_scalar(seeds[j])
    R = (1).to_bytes(32, "little")
    k = o.scalar_from_hash(o.sha512(R + pks[j] + msg))
    ii = list(sigs)
    ii[j] = R + (k * a % o.L).to_bytes(32, "little")
    assert bare.verify_batch([msg] * n, pks, ii, zseed, 3)
    assert not bare.verify_strict(msg, pks[j], ii[j])
    if n <= 67:
        zs = o.batch_coefficients(zseed, 3, n)
        assert o.verify_batch_z([msg] * n, ii, pks, zs)


def test_split_batch_partials(bare):
    """One 667-vote certificate split into 4 shards: the sum of the shards'
    partial points is the identity iff the whole batch verifies; a bad shard flags Err."""
    rng = random.Random(8)
    n = 667
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    msg = bytes(rng.randrange(256) for _ in range(32))
    pks, sigs = bare.sign_many(seeds, [msg] * n)
    zseed = bytes(rng.randrange(256) for _ in range(32))
    cuts = [0, 100, 333, 500, n]

    def split(sg):
        pts, bads = [], []
        for a, b in zip(cuts, cuts[1:]):
            pt, bd = bare.verify_batch_partial([msg] * (b - a), pks[a:b], sg[a:b], zseed, 77, a)
            pts.append(pt)
            bads.append(bd)
        return (not any(bads)) and bare.points_sum_is_identity(pts)

    assert split(sigs) is True
    assert bare.verify_batch([msg] * n, pks, sigs, zseed, 77)
    bad = list(sigs)
    bad[400] = bad[400][:40] + bytes([bad[400][40] ^ 1]) + bad[400][41:]
    assert split(bad) is False
    assert bare.verify_batch([msg] * n, pks, bad, zseed, 77) is False
    hb = list(sigs)
    hb[10] = hb[10][:63] + bytes([hb[10][63] | 0xE0])
    assert split(hb) is False


def test_empty_shards_and_batches(bare):
    """Empty work on the MSM path: a zero-vote shard of a split batch (split_bounds gives
    one whenever the batch has fewer votes than ranks) contributes the identity with no launch
    error, and all-zero or partly-zero counts give dalek's empty-batch verdict, Ok."""
    rng = random.Random(9)
    zseed = bytes(rng.randrange(256) for _ in range(32))
    pt, bad = bare.verify_batch_partial([], [], [], zseed, 3, 0)
    assert not bad and bare.points_sum_is_identity([pt])
    assert bare.verify_batches_pk([0], [], [], [], zseed) == [True]
    assert bare.verify_batches_pk([0, 0, 0], [], [], [], zseed) == [True, True, True]
    n = 5
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    msg = bytes(rng.randrange(256) for _ in range(32))
    pks, sigs = bare.sign_many(seeds, [msg] * n)
    assert bare.verify_batches_pk([0, n, 0], [msg] * n, pks, sigs, zseed) == [True, True, True]
    pts = []
    for a, b in [(0, 0), (0, n), (n, n)]:   # two empty shards around the whole batch
        p, bd = bare.verify_batch_partial([msg] * (b - a), pks[a:b], sigs[a:b], zseed, 4, a)
        assert not bd
        pts.append(p)
    assert bare.points_sum_is_identity(pts)


def test_uncached_then_cached_same_verdicts(golden):
    """A key that is verified before and after it enters the cache gets the same verdicts."""
    from narwhal_amd import _lib
    eng = _lib.Engine(device=0, key_window=12)
    try:
        msgs, pks, sigs, want, names = _strict_cases(golden)
        before = eng.verify_strict_many(msgs, pks, sigs)
        bb = _batch_mismatches(eng, golden)
        eng.committee_load(_all_keys(golden))
        after = eng.verify_strict_many(msgs, pks, sigs)
        assert before == after == want and bb == [] and _batch_mismatches(eng, golden) == []
    finally:
        eng.close()
