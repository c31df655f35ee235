"""Small calls' exact path in one workgroup (k_slow_tail): at most TAIL_MAX_CERTS (16) certificates
and SLOW_TAIL_MAX_SIGS (256) signatures run k_slow_prep, k_slow_mul and the certificate tail as
three phases of a single launch; larger calls launch them separately over many workgroups.

The same certificates go through both (the 4-certificate call and the same call with a fifth, clean
certificate appended, which takes it past 256 signatures) and against the oracle, in both message
modes.  70 votes fail the equation with a prime-order component, so the one workgroup's 64 quads
take two passes of z_i D_i; one certificate has an undecodable / changed R and a non-canonical S.
"""
import os

import numpy as np
import pytest

import nw_ref

pytestmark = pytest.mark.gpu

ZSEED = bytes(range(32))
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))
VOTES = 64


@pytest.fixture(scope="module")
def tail_case():
    from narwhal_amd import _lib, workload
    eng = _lib.Engine(device=0)
    com = workload.make_committee(80, eng)
    cs = workload.make_certificates(com, 5, VOTES, eng)
    slots = np.asarray(eng.committee_load_np(com.pks, com.stake), np.uint32)
    sigs = cs.sigs.copy()
    bad = []
    for v in range(60):                          # certificate 0: 60 changed S (SK_BIG terms)
        sigs[v, 40] ^= 1
        bad.append(v)
    for v in range(10):                          # certificate 1: 10 more
        sigs[VOTES + 5 * v, 41] ^= 0x20
        bad.append(VOTES + 5 * v)
    sigs[2 * VOTES + 7, 3] ^= 0x10               # certificate 2: R changed
    sigs[2 * VOTES + 9, 63] |= 0xE0              # ... and S not canonical
    bad += [2 * VOTES + 7, 2 * VOTES + 9]
    yield eng, com, cs, slots, sigs, sorted(bad)
    eng.close()


def _calls(eng, cs, slots, sigs, ncerts):
    nsig = ncerts * VOTES
    first, n = cs.cert_first[:ncerts], cs.cert_n[:ncerts]
    cert = eng.verify_certs_np(first, n, sigs[:nsig], slots[cs.signer[:nsig]], cs.msgs[:ncerts], ZSEED, 0)
    per_sig = np.repeat(cs.msgs[:ncerts], n, axis=0)
    bat = eng.verify_batches_np(first, n, per_sig, slots[cs.signer[:nsig]], sigs[:nsig], ZSEED, 0)
    return cert, bat


def test_one_workgroup_tail_matches_grid_path_and_oracle(tail_case):
    eng, com, cs, slots, sigs, bad = tail_case
    (ok4, sig4, st4), (bok4, bsig4) = _calls(eng, cs, slots, sigs, 4)     # k_slow_tail
    (ok5, sig5, st5), (bok5, bsig5) = _calls(eng, cs, slots, sigs, 5)     # k_slow_prep / mul / finalize
    exp_sig = np.ones(5 * VOTES, bool)
    exp_sig[bad] = False
    assert (sig5.astype(bool) == exp_sig).all() and (bsig5.astype(bool) == exp_sig).all()
    assert (sig4.astype(bool) == exp_sig[:4 * VOTES]).all() and (bsig4.astype(bool) == exp_sig[:4 * VOTES]).all()
    assert list(ok5.astype(bool)) == [False, False, False, True, True]
    assert list(ok4.astype(bool)) == [False, False, False, True]
    assert list(bok4.astype(bool)) == [False, False, False, True] and list(bok5[:4]) == list(bok4)
    assert (st4 == st5[:4]).all()
    import copy
    cs2 = copy.copy(cs)
    cs2.sigs = sigs
    assert nw_ref.verify_certs(cs2, com, [0, 1, 2, 3, 4], ZSEED, THREADS) == [False, False, False, True, True]


def test_one_workgroup_tail_golden_adversarial_batches(golden):
    """Every golden adversarial batch (small-order components, torsion coefficients, mixed R / A /
    S failures) with its keys in the cache is a one-certificate call of at most 256 signatures, so
    the one-workgroup path decides it (tests/test_gpu_keys.py repeats this at every key window)."""
    from narwhal_amd import _lib
    eng = _lib.Engine(device=0)
    try:
        keys = sorted({bytes.fromhex(k) for c in golden["adversarial_batch"] for k, _, _ in c["items"]})
        eng.committee_load(keys)
        bad = []
        for c in golden["adversarial_batch"]:
            items = [(bytes.fromhex(k), bytes.fromhex(s), bytes.fromhex(m)) for k, s, m in c["items"]]
            assert 1 <= len(items) <= 256
            got = eng.verify_batch([m for *_, m in items], [k for k, _, _ in items], [s for _, s, _ in items],
                                   bytes.fromhex(c["zseed"]), c["batch_index"])
            if got != c["ok"]:
                bad.append((c["name"], c["batch_index"]))
        assert not bad, bad
    finally:
        eng.close()
