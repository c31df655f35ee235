"""GPU parity at every BASELINE.json config, on the committee-mode engine the
bench and the Rust shim use (key_window = -1: W20 at 100 keys, W16 at 1,000, W13 at 10,000).

  C2  100 validators, 14,926 certificates x 67 votes (1,000,042 sigs): the benchmarked W20 kernel
  C3  1,000 validators, one round of 1,000 certificates x 667 votes: every certificate vs the oracle
  C5  C3 with 1% adversarial signatures (tests/adversarial_mix.py): every certificate verdict and
      every adversarial strict verdict vs the oracle
  C4  10,000 validators, one GPU's share of a round (1,250 certificates x 6,667 votes, W13)
  W   worker batch digests (worker/src/processor.rs:65): 508,052-B and 1,000,012-B batches

The checker is oracle/nw_ref.c (C restatement of dalek 1.0.1's verify_batch / verify_strict),
pinned against the Python oracle and the golden vectors by the CPU tests.
"""
import hashlib
import os

import numpy as np
import pytest

import nw_ref

pytestmark = pytest.mark.gpu

ZSEED = bytes(range(32))
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


def _engine(window=-1):
    from narwhal_amd import _lib
    return _lib.Engine(device=0, key_window=window)


def _setup(eng, validators, ncerts, votes):
    from narwhal_amd import workload
    com = workload.make_committee(validators, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, ncerts, votes, eng)
    return com, slots, cs


def _verify(eng, cs, slots, zseed=ZSEED, cert_base=0):
    return eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, zseed, cert_base)


# ----------------------------------------------------------------------------- C2 at W20
# Class-scoped engines: each holds up to ~100 GB of key tables, so one config's engine is closed
# before the next one is built.
@pytest.fixture(scope="class")
def c2():
    eng = _engine()
    com, slots, cs = _setup(eng, 100, 14926, 67)
    yield eng, com, slots, cs
    eng.close()


class TestC2W20:
    def test_c2_committee_mode_is_w20(self, c2):
        eng, com, slots, cs = c2
        assert eng.key_window() == 20 and eng.committee_size() == 100
        assert eng.key_negtab()   # 2 x 1.25 x 100 W20 tables fit the budget: the negated copies
        assert cs.nsigs == 1000042

    def test_c2_w20_all_valid(self, c2):
        eng, com, slots, cs = c2
        cert_ok, sig_ok, stake = _verify(eng, cs, slots, os.urandom(32))
        assert cert_ok.all() and sig_ok.all() and (stake == 67).all()
        sel = list(range(0, cs.ncerts, 149))
        assert all(nw_ref.verify_certs(cs, com, sel, ZSEED, THREADS))

    def test_c2_w20_corruptions_vs_oracle(self, c2):
        """Exactly the certificates holding a corrupted vote fail; the per-signature bitmap flags
        exactly the corrupted votes; every failing certificate and 100 passing ones agree with the
        oracle's batch equation under the same coefficients."""
        eng, com, slots, cs0 = c2
        import copy
        cs = copy.copy(cs0)
        rng = np.random.default_rng(3)
        cs.sigs = cs0.sigs.copy()
        bad = rng.choice(cs.nsigs, 300, replace=False)
        kind = rng.integers(0, 3, size=bad.shape[0])
        for b, k in zip(bad, kind):
            if k == 0:
                cs.sigs[b, 40] ^= 1
            elif k == 1:
                cs.sigs[b, 3] ^= 0x10
            else:
                cs.sigs[b, 63] |= 0xE0
        cert_ok, sig_ok, stake = _verify(eng, cs, slots)
        exp_sig = np.ones(cs.nsigs, bool)
        exp_sig[bad] = False
        assert (sig_ok.astype(bool) == exp_sig).all()
        bad_certs = sorted(set((bad // 67).tolist()))
        exp_cert = np.ones(cs.ncerts, bool)
        exp_cert[bad_certs] = False
        assert (cert_ok.astype(bool) == exp_cert).all()
        # every certificate of the C2 set against the oracle (1,000,042 signatures on the host threads)
        sel = list(range(cs.ncerts))
        want = nw_ref.verify_certs(cs, com, sel, ZSEED, THREADS)
        assert [bool(cert_ok[c]) for c in sel] == want
        assert [int(stake[c]) for c in bad_certs] == [67 - int((bad // 67 == c).sum()) for c in bad_certs]

    def test_c2_w20_device_path_matches_host_path(self, c2):
        """nw_verify_certs_dev (the benchmarked entry point) on HBM-resident inputs, asynchronous
        status word: same verdicts and flags as the host-buffer path."""
        import torch
        eng, com, slots, cs = c2
        dev = torch.device("cuda", 0)
        sigs = cs.sigs.copy()
        sigs[5, 40] ^= 1
        d_sig = torch.from_numpy(sigs).to(dev)
        d_signer = torch.from_numpy(slots[cs.signer].astype(np.int32)).to(dev)
        d_first = torch.from_numpy(cs.cert_first.astype(np.int32)).to(dev)
        d_n = torch.from_numpy(cs.cert_n.astype(np.int32)).to(dev)
        d_msg = torch.from_numpy(cs.msgs).to(dev)
        d_ok = torch.zeros(cs.ncerts, dtype=torch.uint8, device=dev)
        d_flags = torch.zeros(cs.nsigs, dtype=torch.int32, device=dev)
        d_stake = torch.zeros(cs.ncerts, dtype=torch.int64, device=dev)
        d_status = torch.full((1,), 77, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream()
        eng.verify_certs_dev(cs.ncerts, d_first.data_ptr(), d_n.data_ptr(), cs.nsigs, d_sig.data_ptr(),
                             d_signer.data_ptr(), d_msg.data_ptr(), ZSEED, 0, d_ok.data_ptr(), d_flags.data_ptr(),
                             d_stake.data_ptr(), st.cuda_stream, d_status=d_status.data_ptr())
        torch.cuda.synchronize()
        assert int(d_status.item()) == 0
        import copy
        cs2 = copy.copy(cs)
        cs2.sigs = sigs
        cert_ok, sig_ok, stake = _verify(eng, cs2, slots)
        assert (d_ok.cpu().numpy() == cert_ok).all()
        assert ((d_flags.cpu().numpy() & 0x8 != 0) == sig_ok.astype(bool)).all()
        assert (d_stake.cpu().numpy() == stake.astype(np.int64)).all()
        assert not cert_ok[0] and cert_ok[1:].all()


# ----------------------------------------------------------------------------- C1
def test_c1_every_certificate_vs_oracle():
    """BASELINE configs[0] at full size: a 4-validator committee (quorum 3), 10,000 certificates x 3
    votes.  200 votes are corrupted (flipped R bit, S >= 2^253, another message); every certificate's
    batch verdict and accepted stake, and every vote's strict verdict, against the oracle."""
    import ed25519_oracle as o
    eng = _engine()
    try:
        com, slots, cs = _setup(eng, 4, 10000, 3)
        assert cs.nsigs == 30000 and eng.committee_size() == 4
        rng = np.random.default_rng(41)
        bad = rng.choice(cs.nsigs, 200, replace=False)
        sigs = cs.sigs.copy()
        cert_of = np.repeat(np.arange(cs.ncerts), 3)
        for j, b in enumerate(bad):
            if j % 3 == 0:
                sigs[b, 5] ^= 0x20
            elif j % 3 == 1:
                sigs[b, 63] |= 0xE0
            else:
                sigs[b] = np.frombuffer(o.sign(bytes(com.seeds[cs.signer[b]]), bytes(cs.msgs[cert_of[b]])[::-1]),
                                        np.uint8)
        import copy
        cs2 = copy.copy(cs)
        cs2.sigs = sigs
        for base in (0, 20000):
            cert_ok, sig_ok, stake = _verify(eng, cs2, slots, ZSEED, base)
            want = nw_ref.verify_certs(cs2, com, list(range(cs.ncerts)), ZSEED, THREADS, cert_base=base)
            assert cert_ok.astype(bool).tolist() == want
        exp = np.ones(cs.nsigs, bool)
        exp[bad] = False
        assert (sig_ok.astype(bool) == exp).all()
        assert [bool(sig_ok[b]) for b in bad[:30]] == [nw_ref.verify_strict(bytes(com.pks[cs.signer[b]]),
                                                                          bytes(cs.msgs[cert_of[b]]), bytes(sigs[b]))
                                                      for b in bad[:30]]
        assert (stake == np.bincount(cert_of, weights=exp.astype(np.int64), minlength=cs.ncerts)).all()
    finally:
        eng.close()


# ----------------------------------------------------------------------------- C3 / C5
@pytest.fixture(scope="class")
def c3():
    eng = _engine()
    com, slots, cs = _setup(eng, 1000, 1000, 667)
    yield eng, com, slots, cs
    eng.close()


class TestC3C5:
    def test_c3_every_certificate_vs_oracle(self, c3):
        eng, com, slots, cs = c3
        assert eng.key_window() == 16 and cs.nsigs == 667000
        cert_ok, sig_ok, stake = _verify(eng, cs, slots)
        want = nw_ref.verify_certs(cs, com, list(range(cs.ncerts)), ZSEED, THREADS)
        assert cert_ok.astype(bool).tolist() == want
        assert all(want) and sig_ok.all() and (stake == 667).all()

    def test_c5_adversarial_mix_vs_oracle(self, c3):
        """1% of the C3 signatures replaced by classes (ii)/(iii)/(v)/(vi)/(vii)/(viii)/(ix): every
        certificate's batch verdict and every adversarial signature's strict verdict match the oracle
        (nearly every certificate takes the per-signature fallback)."""
        import copy
        from adversarial_mix import make_adversarial
        eng, com, slots, cs0 = c3
        cs = copy.copy(cs0)
        kinds = make_adversarial(cs, com, 0.01, np.random.default_rng(5))
        assert len(kinds) == 6670
        for base in (0, 7000):   # two coefficient streams: the torsion classes depend on z
            cert_ok, sig_ok, stake = _verify(eng, cs, slots, ZSEED, base)
            want = nw_ref.verify_certs(cs, com, list(range(cs.ncerts)), ZSEED, THREADS, cert_base=base)
            got = cert_ok.astype(bool).tolist()
            assert got == want, [c for c in range(cs.ncerts) if got[c] != want[c]][:10]
        cert_of = np.repeat(np.arange(cs.ncerts), cs.cert_n.astype(np.int64))
        bad = []
        for i, cls in kinds.items():
            w = nw_ref.verify_strict(bytes(com.pks[cs.signer[i]]), bytes(cs.msgs[cert_of[i]]), bytes(cs.sigs[i]))
            if bool(sig_ok[i]) != w:
                bad.append((i, cls))
        assert not bad, bad[:10]
        honest = np.ones(cs.nsigs, bool)
        honest[list(kinds)] = False
        assert sig_ok[honest].all()
        # accepted stake counts exactly the strictly valid votes
        exp_stake = np.bincount(cert_of, weights=sig_ok.astype(np.int64), minlength=cs.ncerts)
        assert (stake == exp_stake).all()

    def test_c5_key_classes_at_committee_scale_vs_oracle(self, c3):
        """The full C5 mix including the key-level classes: 2 committee members hold small-order
        keys (class i) and 3 hold mixed-order keys aB + jT8 (class iv), all five loaded into the key
        cache next to the 1,000 honest keys, plus the 1% signature-level mix.  ~3,300 votes come
        from the torsion keys; every certificate verdict (two coefficient streams: the torsion
        coefficients depend on z), every non-honest strict verdict and the accepted stake match
        the oracle."""
        import copy
        from adversarial_mix import add_torsion_members, make_adversarial
        eng, com0, slots0, cs0 = c3
        cs = copy.copy(cs0)
        com, kinds = add_torsion_members(cs, com0, [17, 503], [42, 311, 777])
        assert len(kinds) == 5 * 667
        new_slots = eng.committee_load_np(com.pks[com0.size:], com.stake[com0.size:])
        assert eng.key_window() == 16
        slots = np.concatenate([slots0, np.asarray(new_slots, slots0.dtype)])
        kinds.update(make_adversarial(cs, com, 0.01, np.random.default_rng(11)))
        for base in (0, 7000):
            cert_ok, sig_ok, stake = _verify(eng, cs, slots, ZSEED, base)
            want = nw_ref.verify_certs(cs, com, list(range(cs.ncerts)), ZSEED, THREADS, cert_base=base)
            got = cert_ok.astype(bool).tolist()
            assert got == want, [c for c in range(cs.ncerts) if got[c] != want[c]][:10]
        assert 0 < sum(want) < cs.ncerts
        cert_of = np.repeat(np.arange(cs.ncerts), cs.cert_n.astype(np.int64))
        bad = [(i, cls) for i, cls in kinds.items()
               if bool(sig_ok[i]) != nw_ref.verify_strict(bytes(com.pks[cs.signer[i]]), bytes(cs.msgs[cert_of[i]]),
                                                          bytes(cs.sigs[i]))]
        assert not bad, bad[:10]
        assert not any(sig_ok[i] for i, cls in kinds.items() if cls == "i")   # small-order A: strict rejects
        honest = np.ones(cs.nsigs, bool)
        honest[list(kinds)] = False
        assert sig_ok[honest].all()
        exp_stake = np.bincount(cert_of, weights=sig_ok.astype(np.int64), minlength=cs.ncerts)
        assert (stake == exp_stake).all()


    def test_c5_rank_shards_match_one_call_and_oracle(self, c3):
        """multi-rank verdict identity on the real engine.  The C5 classes (0.1%
        signature-level classes plus the torsion committee keys, whose batch verdicts depend on z)
        is cut into world = 2 and 8 rank shards exactly as shard.verify_sharded and bench.py cut it
        (shard.partition, per-shard arrays, cert_base = global base + c0).  Each rank's shard runs
        through the library on the host path (nw_verify_certs, shard.verify_shard) and on the
        device path bench.py times (nw_verify_certs_dev with a status word); the concatenated
        verdicts and stake equal the one-call result and the oracle, for two coefficient streams."""
        import copy
        import torch
        from adversarial_mix import add_torsion_members, make_adversarial
        from narwhal_amd import shard
        eng, com0, slots0, cs0 = c3
        cs = copy.copy(cs0)
        com, _ = add_torsion_members(cs, com0, [17, 503], [42, 311, 777])
        new_slots = eng.committee_load_np(com.pks[com0.size:], com.stake[com0.size:])
        slots = np.concatenate([slots0, np.asarray(new_slots, slots0.dtype)])
        # 0.1% signature-level classes (667 votes): about half the certificates stay clean, so the
        # concatenated verdicts hold accepts, rejects and torsion-dependent verdicts side by side
        make_adversarial(cs, com, 0.001, np.random.default_rng(23))
        dev = torch.device("cuda", 0)
        stream = torch.cuda.current_stream().cuda_stream
        for base in (0, 7000):
            one_ok, one_sig, one_stake = _verify(eng, cs, slots, ZSEED, base)
            want = nw_ref.verify_certs(cs, com, list(range(cs.ncerts)), ZSEED, THREADS, cert_base=base)
            assert one_ok.astype(bool).tolist() == want
            assert 0 < sum(want) < cs.ncerts
            for world in (2, 8):
                h_ok, h_st, d_ok, d_st, d_strict = [], [], [], [], []
                for rank in range(world):
                    ranges, ok, st = shard.verify_shard(eng, cs, slots, ZSEED, rank, world, base)
                    h_ok.append(ok)
                    h_st.append(st)
                    sh = shard.shard_inputs(cs, slots, rank, world, base)
                    nc, ns = len(sh["n"]), len(sh["sigs"])
                    o_ok = torch.zeros(nc, dtype=torch.uint8, device=dev)
                    o_fl = torch.zeros(ns, dtype=torch.int32, device=dev)
                    o_st = torch.zeros(nc, dtype=torch.int64, device=dev)
                    status = torch.full((1,), 99, dtype=torch.int32, device=dev)
                    t = {k: torch.from_numpy(np.ascontiguousarray(sh[k]).astype(dt)).to(dev)
                         for k, dt in (("first", np.int32), ("n", np.int32), ("sigs", np.uint8),
                                       ("signer_slots", np.int32), ("msgs", np.uint8))}
                    eng.verify_certs_dev(nc, t["first"].data_ptr(), t["n"].data_ptr(), ns, t["sigs"].data_ptr(),
                                         t["signer_slots"].data_ptr(), t["msgs"].data_ptr(), ZSEED, sh["cert_base"],
                                         o_ok.data_ptr(), o_fl.data_ptr(), o_st.data_ptr(), stream,
                                         d_status=status.data_ptr())
                    torch.cuda.synchronize()
                    assert int(status.item()) == 0
                    d_ok.append(o_ok.cpu().numpy())
                    d_st.append(o_st.cpu().numpy())
                    d_strict.append((o_fl.cpu().numpy() & 0x8) != 0)
                assert [r[1] - r[0] for r in ranges] == [len(x) for x in h_ok]
                for got_ok, got_st in ((np.concatenate(h_ok), np.concatenate(h_st)),
                                       (np.concatenate(d_ok), np.concatenate(d_st))):
                    assert (got_ok == one_ok).all(), (base, world, np.flatnonzero(got_ok != one_ok)[:10])
                    assert (got_st.astype(np.int64) == one_stake.astype(np.int64)).all(), (base, world)
                assert (np.concatenate(d_strict) == one_sig.astype(bool)).all(), (base, world)

    def test_split_batch_of_a_6667_vote_certificate(self, c3):
        """VERDICT r04 item 2, split form: ONE 6,667-vote certificate (C4's 2f + 1) split over
        world = 2 and 8 ranks by shard.split_bounds, each rank's row from shard.split_partial_row
        (nw_verify_batch_partial, coefficients at the vote's global index), the verdict from
        shard.split_verdict over the gathered rows (nw_points_sum_is_identity).  Honest, one
        forged vote, and torsion-key votes whose verdict depends on z (eight batch indices): the
        split verdict equals the one-call nw_verify_batch and the oracle every time."""
        import copy
        from adversarial_mix import add_torsion_members
        from narwhal_amd import shard, workload
        eng = c3[0]
        com0 = workload.make_committee(6667, eng)   # not all cached (the C3 keys are its first 1,000): MSM path
        cs0 = workload.make_certificates(com0, 1, 6667, eng)
        msgs = [bytes(cs0.msgs[0])] * 6667
        zseed = bytes(range(40, 72))

        def case(cs, com, bi):
            pks = [bytes(com.pks[k]) for k in cs.signer]
            sigs = [bytes(x) for x in cs.sigs]
            one = eng.verify_batch(msgs, pks, sigs, zseed, bi)
            want = nw_ref.verify_batch_msgs(msgs, pks, sigs, zseed, bi)
            assert one == want, bi
            for world in (2, 8):
                rows = [shard.split_partial_row(eng, msgs, pks, sigs, zseed, bi, r, world) for r in range(world)]
                assert shard.split_verdict(eng, rows) == want, (bi, world)
            return want

        assert case(cs0, com0, 5) is True
        forged = copy.copy(cs0)
        forged.sigs = cs0.sigs.copy()
        forged.sigs[3333] = np.frombuffer(nw_ref_sign_other(com0, cs0, 3333), np.uint8)
        assert case(forged, com0, 5) is False
        tors = copy.copy(cs0)
        com_t, kinds = add_torsion_members(tors, com0, [], [100, 5000])   # A' = aB + jT8: z-dependent
        assert len(kinds) == 2
        verdicts = [case(tors, com_t, bi) for bi in range(8)]
        print("torsion-key split verdicts over 8 batch indices:", verdicts)


def nw_ref_sign_other(com, cs, i):
    """Vote i re-signed over another message (class ix: valid encodings, wrong equation)."""
    import ed25519_oracle as o
    return o.sign(bytes(com.seeds[cs.signer[i]]), bytes(cs.msgs[0])[::-1])


# ----------------------------------------------------------------------------- C4
def test_c4_w13_every_certificate_vs_oracle_and_localized():
    eng = _engine()
    try:
        com, slots, cs = _setup(eng, 10000, 1250, 6667)
        assert eng.key_window() == 13 and cs.nsigs == 1250 * 6667
        rng = np.random.default_rng(9)
        bad = rng.choice(cs.nsigs, 40, replace=False)
        sigs = cs.sigs
        orig = sigs[bad].copy()
        sigs[bad, 40] ^= 1
        cert_ok, sig_ok, stake = _verify(eng, cs, slots)
        exp_sig = np.ones(cs.nsigs, bool)
        exp_sig[bad] = False
        assert (sig_ok.astype(bool) == exp_sig).all()
        bad_certs = sorted(set((bad // 6667).tolist()))
        exp_cert = np.ones(cs.ncerts, bool)
        exp_cert[bad_certs] = False
        assert (cert_ok.astype(bool) == exp_cert).all()
        # every certificate against the oracle (8,333,750 signatures, Pippenger on the host threads)
        sel = list(range(cs.ncerts))
        assert [bool(cert_ok[c]) for c in sel] == nw_ref.verify_certs(cs, com, sel, ZSEED, THREADS)
        assert [int(stake[c]) for c in bad_certs] == [6667 - int((bad // 6667 == c).sum()) for c in bad_certs]
        sigs[bad] = orig
    finally:
        eng.close()


# ----------------------------------------------------------------------------- worker digests
@pytest.mark.parametrize("n_tx,tx_size", [(977, 512), (62500, 8)])
def test_worker_batch_digests_vs_hashlib(engine, n_tx, tx_size):
    """SHA512(bincode WorkerMessage::Batch) of 508,052-B (512-B tx) and 1,000,012-B (8-B tx)
    batches, 16 of each at once, plus one lone batch."""
    from narwhal_amd import workload
    host = workload.worker_batches_np(16, n_tx, tx_size)
    assert host.shape[1] == 12 + n_tx * (8 + tx_size)
    assert bytes(host[3]) == workload.worker_batch(n_tx, tx_size, 3)
    got = engine.sha512_many([bytes(b) for b in host])
    assert got == [hashlib.sha512(bytes(b)).digest() for b in host]
    assert engine.sha512(bytes(host[0])) == hashlib.sha512(bytes(host[0])).digest()



def test_sha512_many_mixed_lengths_unaligned(engine):
    """k_sha512_many on mixed lengths (empty, sub-block, 111/112/128-B boundaries, a worker batch)
    at unaligned offsets, through the device entry point, vs hashlib."""
    import torch
    rng = np.random.default_rng(17)
    lens = [0, 1, 111, 112, 127, 128, 129, 239, 240, 255, 256, 5000, 70001, 508052] + \
        [int(x) for x in rng.integers(0, 20000, size=120)]
    msgs = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in lens]
    offs, pos = [], 3                  # start unaligned
    for m in msgs:
        offs.append(pos)
        pos += len(m) + int(rng.integers(0, 5))
    blob = np.zeros(pos + 16, np.uint8)
    for o, m in zip(offs, msgs):
        blob[o:o + len(m)] = np.frombuffer(m, np.uint8)
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(blob).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int64, device=dev)
    d_out = torch.zeros((len(msgs), 64), dtype=torch.uint8, device=dev)
    engine.sha512_many_dev(d_blob.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(msgs), d_out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    bad = [i for i, m in enumerate(msgs) if bytes(got[i]) != hashlib.sha512(m).digest()]
    assert not bad, [(i, lens[i]) for i in bad[:10]]


def test_sha512_many_33_groups_mixed_lengths(engine):
    """k_sha512_split2 on 33 groups of 32 messages (an exclusive-CU launch: >= 8 workgroups) with mixed
    lengths, so the groups end after different block counts and one group is partial; unaligned
    offsets; vs hashlib.  (Round 6 A/B'd two groups per workgroup on this shape: rejected,
    profiles/r06/c4_digest_packing_ab_r06.txt.)"""
    import torch
    rng = np.random.default_rng(23)
    n = 32 * 32 + 5
    lens = [0, 1, 111, 112, 127, 128, 129, 239, 240, 255, 256, 5000] + \
        [int(x) for x in rng.integers(0, 9000, size=n - 13)] + [70001]
    msgs = [rng.integers(0, 256, size=k, dtype=np.uint8).tobytes() for k in lens]
    offs, pos = [], 5
    for m in msgs:
        offs.append(pos)
        pos += len(m) + int(rng.integers(0, 5))
    blob = np.zeros(pos + 16, np.uint8)
    for o, m in zip(offs, msgs):
        blob[o:o + len(m)] = np.frombuffer(m, np.uint8)
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(blob).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int64, device=dev)
    d_out = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    engine.sha512_many_dev(d_blob.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    bad = [i for i, m in enumerate(msgs) if bytes(got[i]) != hashlib.sha512(m).digest()]
    assert not bad, [(i, lens[i]) for i in bad[:10]]


# ----------------------------------------------------------------------------- C4 headers
def test_c4_headers_with_6667_parents():
    """(f)2 at the size that motivates it: at N = 10,000 a header carries 2f+1 = 6,667 parents, so
    Header::verify rehashes a 213,392-B preimage (primary/src/messages.rs:50, preimage :71-83) before
    the certificate's 6,667-vote batch.  Through verify_certificates (Python orchestration) and the
    native frame path (nw_certificates_verify): header digests vs hashlib, batch verdicts vs the C
    oracle, and the reference's error order (InvalidHeaderId before the signatures)."""
    import time
    import hashlib as hl
    from narwhal_amd import primary as pm
    from narwhal_amd import workload
    eng = _engine()
    try:
        wc = workload.make_committee(10000, eng)
        keys = [bytes(k) for k in wc.pks]
        seed_of = {bytes(k): bytes(s) for k, s in zip(wc.pks, wc.seeds)}
        com = pm.Committee({k: (1, [0]) for k in keys})
        assert com.quorum_threshold() == 6667
        order = com.keys()
        rng = np.random.default_rng(21)
        certs = []
        for r in range(4):
            author = order[r * 13]
            parents = [rng.bytes(32) for _ in range(6667)]
            h = pm.Header(author, r + 1, {}, parents)
            pre = h.digest_preimage()
            assert len(pre) == 32 + 8 + 6667 * 32
            h.id = hl.sha512(pre).digest()[:32]
            _, hs = eng.sign_many_np(np.frombuffer(seed_of[author], np.uint8).reshape(1, 32),
                                     np.frombuffer(h.id, np.uint8).reshape(1, 32))
            h.signature = bytes(hs[0])
            voters = [order[(r * 101 + k) % 10000] for k in range(6667)]
            d = hl.sha512(pm.Vote(h.id, h.round, h.author, keys[0]).digest_preimage()).digest()[:32]
            _, vs = eng.sign_many_np(np.stack([np.frombuffer(seed_of[v], np.uint8) for v in voters]),
                                     np.tile(np.frombuffer(d, np.uint8), (6667, 1)))
            certs.append(pm.Certificate(h, [(v, bytes(s)) for v, s in zip(voters, vs)]))
        # cert 1: one parent byte changed after signing -> InvalidHeaderId; cert 2: one bad vote
        p0 = sorted(certs[1].header.parents)[3000]
        certs[1].header.parents.discard(p0)
        certs[1].header.parents.add(bytes([p0[0] ^ 1]) + p0[1:])
        k, s = certs[2].votes[4321]
        certs[2].votes[4321] = (k, s[:40] + bytes([s[40] ^ 2]) + s[41:])
        # GPU digests of the 213 KB preimages == hashlib
        pres = [c.header.digest_preimage() for c in certs]
        assert eng.sha512_many(pres) == [hl.sha512(p).digest() for p in pres]
        zseed = bytes([3]) * 32
        t0 = time.perf_counter()
        got = pm.verify_certificates(certs, com, eng, zseed=zseed, cert_base=40)
        t_py = time.perf_counter() - t0
        frames = [pm.encode_primary_message(c) for c in certs]
        t0 = time.perf_counter()
        native = pm.verify_certificate_frames(frames, com, eng, zseed=zseed, cert_base=40)
        t_nat = time.perf_counter() - t0
        want_types = [None, pm.InvalidHeaderId, pm.InvalidSignature, None]
        assert [type(e) if e else None for e in got] == want_types
        assert [type(e) if e else None for e in native] == want_types
        # the batch step vs the C oracle for the certificates that reach it (batch index = order
        # among the certificates that reach the batch step, as nw_cert_batch_verify numbers them)
        reach = [0, 2, 3]
        for j, ci in enumerate(reach):
            c = certs[ci]
            dg = hl.sha512(c.digest_preimage()).digest()[:32]
            want = nw_ref.crypto_verify_batch(dg, c.votes, zseed, 40 + j)
            assert want == (ci != 2), ci
        # one certificate alone through the native path: the Core::run latency at N = 10,000
        one = pm.verify_certificate_frames(frames[:1], com, eng, zseed=zseed)
        assert one == [None]
        print("\n6,667-parent headers: 4 certs verify_certificates %.1f ms, native %.1f ms" % (t_py * 1e3,
                                                                                         t_nat * 1e3))
    finally:
        eng.close()


def test_sha512_throughput_kernel_many_messages(engine):
    """More messages than the schedule/round split serves (> 32,768: k_sha512_many, one lane per
    message, 4+ waves per SIMD): mixed lengths across the 111/112/128-byte padding boundaries at
    unaligned offsets, vs hashlib."""
    import torch
    rng = np.random.default_rng(23)
    n = 40000
    lens = rng.integers(0, 700, size=n)
    lens[:8] = [0, 111, 112, 127, 128, 129, 239, 256]
    offs = np.zeros(n, np.int64)
    pos = 1
    for i in range(n):
        offs[i] = pos
        pos += int(lens[i]) + int(rng.integers(0, 4))
    blob = rng.integers(0, 256, size=pos + 8, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(blob).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int64)).to(dev)
    d_out = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    engine.sha512_many_dev(d_blob.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    bad = [i for i in range(n)
           if bytes(got[i]) != hashlib.sha512(blob[offs[i]:offs[i] + lens[i]].tobytes()).digest()]
    assert not bad, [(i, int(lens[i]), int(offs[i])) for i in bad[:10]]


# ----------------------------------------------------------------------------- large certificates, device ranges
@pytest.mark.parametrize("votes", [300, 1100])
def test_large_certificate_device_ranges(votes):
    """Device-path input checks on certificates large enough for the multi-wave expansion and the
    workgroup finalize (k_expand_count with 2 / 4 waves per certificate, k_cert_finalize_wg<256> /
    <1024>; 20 certificates, above the one-wave tail's 16): two overlapping vote ranges (NW_ERR_ARG
    in the status word, both certificates rejected, neither credited stake it does not own), the
    votes the shifted range left behind (in no certificate: no verdict), a range running past the
    signature array (rejected), a forged vote (rejected, as the oracle says; stake one vote short)
    and honest certificates (accepted with their full stake)."""
    import torch
    eng = _engine()
    try:
        ncerts, last = 20, 19
        com, slots, cs = _setup(eng, votes, ncerts, votes)
        sigs = cs.sigs.copy()
        forged_cert, forged_vote = 1, 7
        i = forged_cert * votes + forged_vote
        sigs[i] = np.frombuffer(nw_ref_sign_other(com, cs, i), np.uint8)
        first = cs.cert_first.astype(np.int64).copy()
        n = cs.cert_n.astype(np.int64).copy()
        first[3] -= 10                      # certificate 3 claims the last 10 votes of certificate 2
        n[last] += 5                        # the last certificate runs past the signature array
        gap = np.arange(4 * votes - 10, 4 * votes)   # certificate 3's own last 10 votes: in no range now
        dev = torch.device("cuda", 0)
        t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in (
            ("first", first.astype(np.int32)), ("n", n.astype(np.int32)), ("sigs", sigs),
            ("signer", slots[cs.signer].astype(np.int32)), ("msgs", cs.msgs))}
        stake_of = np.asarray(com.stake, np.int64)[cs.signer]

        def span(a, b):
            return int(stake_of[a:b].sum())

        want = [c not in (1, 2, 3, last) for c in range(ncerts)]
        for rep in range(3):   # the vote map's atomic order may differ between launches
            ok = torch.full((ncerts,), 7, dtype=torch.uint8, device=dev)
            st = torch.full((ncerts,), -1, dtype=torch.int64, device=dev)
            fl = torch.full((cs.nsigs,), -1, dtype=torch.int32, device=dev)
            status = torch.full((1,), 99, dtype=torch.int32, device=dev)
            eng.verify_certs_dev(ncerts, t["first"].data_ptr(), t["n"].data_ptr(), cs.nsigs, t["sigs"].data_ptr(),
                                 t["signer"].data_ptr(), t["msgs"].data_ptr(), ZSEED, 0, ok.data_ptr(),
                                 fl.data_ptr(), st.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                 d_status=status.data_ptr())
            torch.cuda.synchronize()
            assert int(status.item()) == 2, rep
            assert ok.cpu().numpy().astype(bool).tolist() == want, rep
            stk = st.cpu().numpy()
            for c in range(ncerts):
                if want[c]:
                    assert stk[c] == span(c * votes, (c + 1) * votes), (rep, c)
            assert stk[forged_cert] == span(votes, 2 * votes) - int(stake_of[i]), rep
            # certificate 2 owns its first votes - 10 for sure and the shared 10 if it won them (they
            # verify under its message); certificate 3's shared votes never verify under its message
            assert span(2 * votes, 3 * votes - 10) <= stk[2] <= span(2 * votes, 3 * votes), (rep, stk[2])
            assert stk[3] == span(3 * votes, 4 * votes - 10), (rep, stk[3])
            assert (fl.cpu().numpy()[gap] == 0).all(), rep
        # the forged certificate's verdict from the oracle (its own votes, batch index = its index)
        f0, nv = int(cs.cert_first[forged_cert]), int(cs.cert_n[forged_cert])
        pks = [bytes(com.pks[k]) for k in cs.signer[f0:f0 + nv]]
        assert not nw_ref.verify_batch_msgs([bytes(cs.msgs[forged_cert])] * nv, pks,
                                            [bytes(x) for x in sigs[f0:f0 + nv]], ZSEED, forged_cert)
    finally:
        eng.close()
