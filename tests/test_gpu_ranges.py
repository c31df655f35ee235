"""Certificate vote ranges and digest tails at the edges of the C ABI (round-4 fixes).

* A vote that lies in no certificate's range gets no verdict (sig_ok 0) and never touches a
  certificate's exact-path state.  Before round 4 such a vote was mapped to certificate 0: a bad S
  there doomed certificate 0's exact path (its forged vote could then be accepted), and a forged vote
  there counted as a prime-order term of certificate 0 (an honest certificate 0 was rejected).
* Overlapping vote ranges are NW_ERR_ARG on every entry point (host check, synchronous device check,
  asynchronous status word): a vote's z and exact-path term belong to one certificate.
* The internal NW_F_P_SAVED bit (0x4000) never reaches the caller's flags.
* SHA-512 of unaligned messages whose length mod 128 >= 112 (a padding-only second block) that end
  flush with their buffer: the padding block reads nothing past the message.
Expected verdicts come from the oracle (ed25519-dalek 1.0.1 restated, crypto/src/lib.rs:206-219).
"""
import hashlib
import random

import numpy as np
import pytest

import ed25519_oracle as o

pytestmark = pytest.mark.gpu

ZSEED = bytes(range(1, 33))
NW_F_P_SAVED = 0x4000


@pytest.fixture(scope="module")
def keys(engine):
    rng = random.Random(404)
    seeds = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(7)]
    pks = [o.public_from_seed(s) for s in seeds]
    slots = engine.committee_load(pks, [1] * 7)
    return rng, seeds, pks, slots


def _cert(rng, seeds, n, forge=(), bad_s=()):
    """n votes of keys 0..n-1 over a fresh digest; ``forge``: votes signed over another message
    (valid encoding, wrong equation: a prime-order D), ``bad_s``: votes with S >= 2^253."""
    msg = bytes(rng.randrange(256) for _ in range(32))
    other = bytes(rng.randrange(256) for _ in range(32))
    sigs = []
    for v in range(n):
        s = o.sign(seeds[v], other if v in forge else msg)
        if v in bad_s:
            s = s[:63] + bytes([s[63] | 0xE0])
        sigs.append(s)
    return msg, sigs


def _expect(msg, pks, sigs, cert_index):
    return o.crypto_verify_batch(msg, list(zip(pks, sigs)), ZSEED, cert_index)


@pytest.mark.parametrize("case", ["gap_bad_s_next_to_forged_cert", "gap_forged_next_to_honest_cert",
                                  "leading_gap_bad_s"])
def test_gap_votes_touch_no_certificate(engine, keys, case):
    rng, seeds, pks, slots = keys
    if case == "gap_bad_s_next_to_forged_cert":
        m0, s0 = _cert(rng, seeds, 4, forge=(2,))           # certificate 0: one forged vote
        mg, sg = _cert(rng, seeds, 1, bad_s=(0,))           # gap vote: bad S
    elif case == "gap_forged_next_to_honest_cert":
        m0, s0 = _cert(rng, seeds, 4)                       # certificate 0 honest
        mg, sg = _cert(rng, seeds, 1, forge=(0,))           # gap vote: forged, canonical
    else:
        m0, s0 = _cert(rng, seeds, 4, forge=(1, 3))
        mg, sg = _cert(rng, seeds, 1, bad_s=(0,))
    m1, s1 = _cert(rng, seeds, 5)
    if case == "leading_gap_bad_s":
        sigs = sg + s0 + s1
        certs = [(1, 4), (5, 5)]
        signer = [slots[0]] + slots[:4] + slots[:5]
        gap = [0]
    else:
        sigs = s0 + sg + s1
        certs = [(0, 4), (5, 5)]
        signer = slots[:4] + [slots[0]] + slots[:5]
        gap = [4]
    want = [_expect(m0, pks[:4], s0, 0), _expect(m1, pks[:5], s1, 1)]
    cert_ok, sig_ok, stake = engine.verify_certs(certs, b"".join(sigs), signer, m0 + m1, ZSEED)
    assert cert_ok == want, (case, cert_ok, want)
    assert [sig_ok[g] for g in gap] == [False]
    strict0 = [o.verify_strict(pks[v], m0, s0[v]) for v in range(4)]
    f0 = certs[0][0]
    assert sig_ok[f0:f0 + 4] == strict0
    assert stake == [sum(strict0), 5]
    # the same call through the device path (device preamble, no host-expanded map)
    import torch
    dev = torch.device("cuda", 0)
    d_first = torch.tensor([c[0] for c in certs], dtype=torch.int32, device=dev)
    d_n = torch.tensor([c[1] for c in certs], dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(sigs), np.uint8).copy()).to(dev)
    d_signer = torch.tensor(signer, dtype=torch.int32, device=dev)
    d_msg = torch.from_numpy(np.frombuffer(m0 + m1, np.uint8).copy()).to(dev)
    ok = torch.zeros(2, dtype=torch.uint8, device=dev)
    flags = torch.full((len(sigs),), -1, dtype=torch.int32, device=dev)
    st = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_certs_dev(2, d_first.data_ptr(), d_n.data_ptr(), len(sigs), d_sig.data_ptr(), d_signer.data_ptr(),
                            d_msg.data_ptr(), ZSEED, 0, ok.data_ptr(), flags.data_ptr(), st.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert ok.cpu().numpy().astype(bool).tolist() == want
    fl = flags.cpu().numpy()
    assert [int(fl[g]) for g in gap] == [0]
    assert not (fl & NW_F_P_SAVED).any()
    assert st.cpu().numpy().tolist() == [sum(strict0), 5]


def test_forged_votes_flags_carry_no_internal_bit(engine, keys):
    """Certificates with forged votes (P parked for the exact path): the returned flags hold only
    the documented NW_F_* bits, at a size that takes the device preamble (> 16,384 signatures)."""
    import torch
    rng, seeds, pks, slots = keys
    ncert, nv = 2600, 7
    msgs, sigs = [], []
    for c in range(ncert):
        m, s = _cert(rng, seeds, nv, forge=(c % nv,) if c % 5 == 0 else ())
        msgs.append(m)
        sigs += s
    dev = torch.device("cuda", 0)
    first = np.arange(ncert, dtype=np.int32) * nv
    d_first = torch.from_numpy(first).to(dev)
    d_n = torch.full((ncert,), nv, dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(sigs), np.uint8).copy()).to(dev)
    d_signer = torch.tensor(slots[:nv] * ncert, dtype=torch.int32, device=dev)
    d_msg = torch.from_numpy(np.frombuffer(b"".join(msgs), np.uint8).copy()).to(dev)
    ok = torch.zeros(ncert, dtype=torch.uint8, device=dev)
    flags = torch.zeros(ncert * nv, dtype=torch.int32, device=dev)
    st = torch.zeros(ncert, dtype=torch.int64, device=dev)
    engine.verify_certs_dev(ncert, d_first.data_ptr(), d_n.data_ptr(), ncert * nv, d_sig.data_ptr(),
                            d_signer.data_ptr(), d_msg.data_ptr(), ZSEED, 0, ok.data_ptr(), flags.data_ptr(),
                            st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fl = flags.cpu().numpy()
    assert not (fl & NW_F_P_SAVED).any()
    assert ok.cpu().numpy().astype(bool).tolist() == [c % 5 != 0 for c in range(ncert)]
    for c in (0, 5, 10):   # the forged certificates, against the oracle
        f = c * nv
        assert bool(ok[c].item()) == _expect(msgs[c], pks[:nv], sigs[f:f + nv], c)


def test_overlapping_ranges_are_arg_errors(engine, keys):
    import torch
    from narwhal_amd import _lib
    rng, seeds, pks, slots = keys
    m0, s0 = _cert(rng, seeds, 6)
    certs = [(0, 4), (2, 4)]                               # votes 2 and 3 claimed twice
    with pytest.raises(_lib.DeviceError, match="rc=2"):
        engine.verify_certs(certs, b"".join(s0), slots[:6], m0 + m0, ZSEED)
    with pytest.raises(_lib.DeviceError, match="rc=2"):
        engine.verify_batches([(0, 4), (3, 3)], [m0] * 6, slots[:6], s0, ZSEED)
    # empty ranges overlap nothing; adjacent ranges are fine
    ok, _, _ = engine.verify_certs([(0, 3), (3, 0), (3, 3)], b"".join(s0), slots[:6], m0 * 3, ZSEED)
    assert ok == [_expect(m0, pks[:3], s0[:3], 0), True, _expect(m0, pks[3:6], s0[3:6], 2)]
    dev = torch.device("cuda", 0)
    d_first = torch.tensor([0, 2], dtype=torch.int32, device=dev)
    d_n = torch.tensor([4, 4], dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(s0), np.uint8).copy()).to(dev)
    d_signer = torch.tensor(slots[:6], dtype=torch.int32, device=dev)
    d_msg = torch.from_numpy(np.frombuffer(m0 + m0, np.uint8).copy()).to(dev)
    ok = torch.zeros(2, dtype=torch.uint8, device=dev)
    st = torch.zeros(2, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    args = (2, d_first.data_ptr(), d_n.data_ptr(), 6, d_sig.data_ptr(), d_signer.data_ptr(), d_msg.data_ptr(),
            ZSEED, 0, ok.data_ptr(), 0, st.data_ptr(), stream)
    with pytest.raises(_lib.DeviceError, match="rc=2"):
        engine.verify_certs_dev(*args)
    status = torch.full((1,), 99, dtype=torch.int32, device=dev)
    engine.verify_certs_dev(*args, d_status=status.data_ptr())
    torch.cuda.synchronize()
    assert int(status.item()) == 2
    d_first.copy_(torch.tensor([0, 4], dtype=torch.int32))   # disjoint again: verifies
    d_n.copy_(torch.tensor([4, 2], dtype=torch.int32))
    engine.verify_certs_dev(*args, d_status=status.data_ptr())
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    assert ok.cpu().numpy().astype(bool).tolist() == [_expect(m0, pks[:4], s0[:4], 0),
                                                      _expect(m0, pks[4:6], s0[4:6], 1)]


def test_overlapping_device_ranges_reject_both_certificates(engine, keys):
    """with a device status word the kernels still run on overlapping ranges.
    Votes 0-3 sign m0 (certificate 0 = votes [0, 4)), votes 4-5 sign m1 (certificate 1 = votes
    [2, 6) over m1): votes 2 and 3 are claimed twice, and whichever certificate the vote map ends
    with checks them against ITS message.  Whatever that order, both certificates are rejected and
    neither is credited stake of a vote it does not own."""
    import torch
    rng, seeds, pks, slots = keys
    m0 = bytes(rng.randrange(256) for _ in range(32))
    m1 = bytes(rng.randrange(256) for _ in range(32))
    sigs = [o.sign(seeds[v], m0 if v < 4 else m1) for v in range(6)]
    dev = torch.device("cuda", 0)
    d_first = torch.tensor([0, 2], dtype=torch.int32, device=dev)
    d_n = torch.tensor([4, 4], dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(sigs), np.uint8).copy()).to(dev)
    d_signer = torch.tensor(slots[:6], dtype=torch.int32, device=dev)
    d_msg = torch.from_numpy(np.frombuffer(m0 + m1, np.uint8).copy()).to(dev)
    stream = torch.cuda.current_stream().cuda_stream
    for rep in range(8):   # the atomic order of the vote map may differ from launch to launch
        ok = torch.full((2,), 7, dtype=torch.uint8, device=dev)
        stake = torch.full((2,), -1, dtype=torch.int64, device=dev)
        status = torch.full((1,), 99, dtype=torch.int32, device=dev)
        engine.verify_certs_dev(2, d_first.data_ptr(), d_n.data_ptr(), 6, d_sig.data_ptr(), d_signer.data_ptr(),
                                d_msg.data_ptr(), ZSEED, 0, ok.data_ptr(), 0, stake.data_ptr(), stream,
                                d_status=status.data_ptr())
        torch.cuda.synchronize()
        assert int(status.item()) == 2, rep
        assert ok.cpu().tolist() == [0, 0], rep
        st = stake.cpu().tolist()
        # stake 1 per key.  Certificate 0 owns votes 0-1 for sure and 2-3 if it won them (they match
        # m0); certificate 1 owns 4-5 (match m1) and may own 2-3, which never match m1
        assert 2 <= st[0] <= 4 and st[1] == 2, (rep, st)


@pytest.mark.parametrize("sh", [1, 2, 3])
def test_sha512_unaligned_padding_block_ends_flush(engine, sh):
    """Messages at an odd offset whose length mod 128 >= 112 (the padding needs a second block),
    each ending exactly at the end of its device buffer, through nw_sha512_many_dev."""
    import torch
    dev = torch.device("cuda", 0)
    lens = [112, 120, 127, 128 + 112, 1024 + 125, 16 * 128 + 119]
    rng = np.random.default_rng(sh)
    for L in lens:
        buf = torch.from_numpy(rng.integers(0, 256, sh + L, dtype=np.uint8)).to(dev)   # message = buf[sh:]
        d_off = torch.tensor([sh], dtype=torch.int64, device=dev)
        d_len = torch.tensor([L], dtype=torch.int64, device=dev)
        d_out = torch.zeros((1, 64), dtype=torch.uint8, device=dev)
        engine.sha512_many_dev(buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), 1, d_out.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert bytes(d_out[0].cpu().numpy()) == hashlib.sha512(buf[sh:].cpu().numpy().tobytes()).digest(), L


def _undecodable_r(rng, sig):
    """sig with R replaced by 32 bytes that do not decode (the oracle's decompress fails)."""
    while True:
        r = bytes(rng.randrange(256) for _ in range(32))
        if o.decompress(r) is None:
            return r + sig[32:]


def test_undecodable_r_flags_are_deterministic(engine, keys):
    """Certificates with several undecodable R's: every such vote carries NW_F_R_BAD on every run
    (k_slow_prep decodes each slow entry of a certificate that k_finish did not reject; an R failure
    found in the same kernel no longer makes later entries skip their decode), the certificates are
    rejected, and two runs return identical flags."""
    import torch
    rng, seeds, pks, slots = keys
    ncert, nv = 300, 7
    msgs, sigs, bad = [], [], set()
    for c in range(ncert):
        m, s = _cert(rng, seeds, nv)
        if c % 3 == 0:
            for v in (1, 3, 5):
                s[v] = _undecodable_r(rng, s[v])
                bad.add(c * nv + v)
        msgs.append(m)
        sigs += s
    dev = torch.device("cuda", 0)
    d_first = torch.from_numpy(np.arange(ncert, dtype=np.int32) * nv).to(dev)
    d_n = torch.full((ncert,), nv, dtype=torch.int32, device=dev)
    d_sig = torch.from_numpy(np.frombuffer(b"".join(sigs), np.uint8).copy()).to(dev)
    d_signer = torch.tensor(slots[:nv] * ncert, dtype=torch.int32, device=dev)
    d_msg = torch.from_numpy(np.frombuffer(b"".join(msgs), np.uint8).copy()).to(dev)
    runs = []
    for _ in range(3):
        ok = torch.zeros(ncert, dtype=torch.uint8, device=dev)
        flags = torch.zeros(ncert * nv, dtype=torch.int32, device=dev)
        st = torch.zeros(ncert, dtype=torch.int64, device=dev)
        engine.verify_certs_dev(ncert, d_first.data_ptr(), d_n.data_ptr(), ncert * nv, d_sig.data_ptr(),
                                d_signer.data_ptr(), d_msg.data_ptr(), ZSEED, 0, ok.data_ptr(), flags.data_ptr(),
                                st.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        runs.append((ok.cpu().numpy().astype(bool), flags.cpu().numpy()))
    ok0, fl0 = runs[0]
    for okr, flr in runs[1:]:
        assert (okr == ok0).all() and (flr == fl0).all()
    assert ok0.tolist() == [c % 3 != 0 for c in range(ncert)]
    r_bad = {int(i) for i in np.nonzero(fl0 & 0x2000)[0]}
    assert r_bad == bad
    for c in (0, 3, 1):
        f = c * nv
        assert bool(ok0[c]) == _expect(msgs[c], pks[:nv], sigs[f:f + nv], c)
