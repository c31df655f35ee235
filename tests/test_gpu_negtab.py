"""Key tables with and without their negated copies (nw_key_negtab): k_verify<MSGMODE, WA, NT>
reads a signed digit's entry from T+ or T- by address when the copies exist, and negates T+ entries
in the addition when they do not (nw_opts.flags NW_OPT_NO_KEY_NEGTAB, or a cache too large for twice
the tables).  Both kernels, in both message modes, must give the oracle's verdicts bit for bit.

40,200 signatures per call: above VERIFY_SPLIT_MAX_SIGS (16,384), so the throughput kernel runs,
not the latency split kernel.
"""
import os

import numpy as np
import pytest

import nw_ref

pytestmark = pytest.mark.gpu

ZSEED = bytes(range(32))
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))
VALIDATORS, NCERTS, VOTES = 200, 600, 67


@pytest.fixture(scope="module")
def workload_200():
    from narwhal_amd import _lib, workload
    eng = _lib.Engine(device=0)
    com = workload.make_committee(VALIDATORS, eng)
    cs = workload.make_certificates(com, NCERTS, VOTES, eng)
    eng.close()
    rng = np.random.default_rng(11)
    sigs = cs.sigs.copy()
    bad = rng.choice(cs.nsigs, 120, replace=False)
    for j, b in enumerate(bad):
        if j % 3 == 0:
            sigs[b, 40] ^= 1          # S changed: the equation fails
        elif j % 3 == 1:
            sigs[b, 3] ^= 0x10        # R changed
        else:
            sigs[b, 63] |= 0xE0       # S not canonical
    return com, cs, sigs, bad


def _run(negtab, window, com, cs, sigs):
    from narwhal_amd import _lib
    eng = _lib.Engine(device=0, key_window=window, flags=0 if negtab else _lib.NW_OPT_NO_KEY_NEGTAB)
    try:
        slots = np.asarray(eng.committee_load_np(com.pks, com.stake), np.uint32)
        assert eng.key_negtab() == negtab and eng.key_window() == window
        cert = eng.verify_certs_np(cs.cert_first, cs.cert_n, sigs, slots[cs.signer], cs.msgs, ZSEED, 0)
        # MSGMODE 1 (per-signature messages): each vote's message is its certificate digest
        per_sig = np.repeat(cs.msgs, cs.cert_n, axis=0)
        bat = eng.verify_batches_np(cs.cert_first, cs.cert_n, per_sig, slots[cs.signer], sigs, ZSEED, 0)
    finally:
        eng.close()
    return cert, bat


@pytest.mark.parametrize("window", [12, 16])
def test_negtab_and_plain_tables_match_oracle(workload_200, window):
    com, cs, sigs, bad = workload_200
    (ok1, sig1, st1), (bok1, bsig1) = _run(True, window, com, cs, sigs)
    (ok0, sig0, st0), (bok0, bsig0) = _run(False, window, com, cs, sigs)
    exp_sig = np.ones(cs.nsigs, bool)
    exp_sig[bad] = False
    exp_cert = np.ones(cs.ncerts, bool)
    exp_cert[sorted(set((bad // VOTES).tolist()))] = False
    for sig_ok in (sig1, sig0, bsig1, bsig0):
        assert (sig_ok.astype(bool) == exp_sig).all()
    for cert_ok in (ok1, ok0, bok1, bok0):
        assert (cert_ok.astype(bool) == exp_cert).all()
    assert (st1 == st0).all()
    # the batch equation itself against the oracle, same coefficients
    import copy
    cs2 = copy.copy(cs)
    cs2.sigs = sigs
    sel = list(range(0, cs.ncerts, 7)) + sorted(set((bad // VOTES).tolist()))
    want = nw_ref.verify_certs(cs2, com, sel, ZSEED, THREADS)
    assert [bool(ok1[c]) for c in sel] == want


def test_shared_basepoint_table_outlives_the_first_context(workload_200):
    """The basepoint comb is shared by the contexts of a process on a device (reference-counted):
    a second engine verifies correctly while the first is alive and after the first is closed."""
    from narwhal_amd import _lib
    com, cs, sigs, bad = workload_200
    sel = slice(0, 64)
    first = np.asarray(cs.cert_first[sel], np.uint32)
    n = np.asarray(cs.cert_n[sel], np.uint32)
    nsig = int(first[-1] + n[-1])
    e1 = _lib.Engine(device=0, key_window=12)
    e2 = _lib.Engine(device=0, key_window=12)
    try:
        s1 = np.asarray(e1.committee_load_np(com.pks, com.stake), np.uint32)
        s2 = np.asarray(e2.committee_load_np(com.pks, com.stake), np.uint32)
        want = np.ones(len(n), bool)
        want[sorted({int(b) // VOTES for b in bad if b < nsig})] = False
        ok1, _, _ = e1.verify_certs_np(first, n, sigs[:nsig], s1[cs.signer[:nsig]], cs.msgs[sel], ZSEED, 0)
        ok2, _, _ = e2.verify_certs_np(first, n, sigs[:nsig], s2[cs.signer[:nsig]], cs.msgs[sel], ZSEED, 0)
        assert (ok1.astype(bool) == want).all() and (ok2.astype(bool) == want).all()
        e1.close()
        ok3, _, _ = e2.verify_certs_np(first, n, sigs[:nsig], s2[cs.signer[:nsig]], cs.msgs[sel], ZSEED, 0)
        assert (ok3.astype(bool) == want).all()
        e3 = _lib.Engine(device=0, key_window=12)   # re-acquires the live table
        s3 = np.asarray(e3.committee_load_np(com.pks, com.stake), np.uint32)
        ok4, _, _ = e3.verify_certs_np(first, n, sigs[:nsig], s3[cs.signer[:nsig]], cs.msgs[sel], ZSEED, 0)
        assert (ok4.astype(bool) == want).all()
        e3.close()
    finally:
        e2.close()
        e1.close()


def test_auto_window_never_takes_negated_copies(workload_200):
    """an automatic window (nw_opts.key_window 0: keys added over time, no declared
    bound) keeps single tables, so its key capacity is not halved by T-; an explicit window on the same
    keys takes T- (2.9 GB of W12 tables).  Verdicts on both equal the oracle's (the workload's
    corrupted votes)."""
    from narwhal_amd import _lib
    com, cs, sigs, bad = workload_200
    sel = slice(0, 64)
    first = np.asarray(cs.cert_first[sel], np.uint32)
    n = np.asarray(cs.cert_n[sel], np.uint32)
    nsig = int(first[-1] + n[-1])
    want = np.ones(len(n), bool)
    want[sorted({int(b) // VOTES for b in bad if b < nsig})] = False
    for window, negtab in ((0, False), (12, True)):
        eng = _lib.Engine(device=0, key_window=window)
        try:
            s = np.asarray(eng.committee_load_np(com.pks, com.stake), np.uint32)
            assert eng.key_negtab() == negtab, (window, eng.key_window())
            ok, _, _ = eng.verify_certs_np(first, n, sigs[:nsig], s[cs.signer[:nsig]], cs.msgs[sel], ZSEED, 0)
            assert (ok.astype(bool) == want).all()
        finally:
            eng.close()
