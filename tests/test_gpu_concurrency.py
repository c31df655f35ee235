"""Reentrancy and input validation of the C ABI (the worker calls from 64 rayon
threads, worker/src/processor.rs:75-79).

* Several threads call nw_verify_certs_dev (each on its own HIP stream), nw_verify_certs (host
  buffers) and the uncached-key paths on ONE context at the same time; every verdict equals the
  serial result, which is itself checked against the oracle.
* nw_verify_certs_dev with a signer slot outside the key cache or a vote range past nsigs returns
  NW_ERR_ARG (synchronous check) or writes NW_ERR_ARG to the status word (asynchronous), and never
  faults.
* A NULL zseed is NW_ERR_ARG at every batch entry point.
* One thread with batches in flight on three streams (bench.py --streams 3): calls alternate between
  the streams with no synchronization in between, each on its own workspace, every output set
  equals the serial result, and repeated calls return identical flag words.
"""
import ctypes
import threading

import numpy as np
import pytest

import nw_ref

pytestmark = pytest.mark.gpu

ZSEED = bytes(range(32))


@pytest.fixture(scope="module")
def setup():
    import torch
    from narwhal_amd import _lib, workload
    eng = _lib.Engine(device=0, key_window=16)
    com = workload.make_committee(40, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, 600, 27, eng)
    sigs = cs.sigs.copy()
    rng = np.random.default_rng(12)
    bad = rng.choice(cs.nsigs, 25, replace=False)
    sigs[bad, 41] ^= 2
    cs.sigs = sigs
    dev = torch.device("cuda", 0)
    yield eng, com, slots, cs, dev
    eng.close()


def _dev_inputs(cs, slots, dev):
    import torch
    return dict(sig=torch.from_numpy(cs.sigs).to(dev),
                signer=torch.from_numpy(slots[cs.signer].astype(np.int32)).to(dev),
                first=torch.from_numpy(cs.cert_first.astype(np.int32)).to(dev),
                n=torch.from_numpy(cs.cert_n.astype(np.int32)).to(dev),
                msg=torch.from_numpy(cs.msgs).to(dev))


def _run_dev(eng, cs, d, dev, stream, cert_base, status=None):
    import torch
    ok = torch.zeros(cs.ncerts, dtype=torch.uint8, device=dev)
    flags = torch.zeros(cs.nsigs, dtype=torch.int32, device=dev)
    stake = torch.zeros(cs.ncerts, dtype=torch.int64, device=dev)
    eng.verify_certs_dev(cs.ncerts, d["first"].data_ptr(), d["n"].data_ptr(), cs.nsigs, d["sig"].data_ptr(),
                         d["signer"].data_ptr(), d["msg"].data_ptr(), ZSEED, cert_base, ok.data_ptr(),
                         flags.data_ptr(), stake.data_ptr(), stream.cuda_stream,
                         d_status=None if status is None else status.data_ptr())
    return ok, flags, stake


def test_concurrent_dev_host_and_uncached_calls(setup):
    import torch
    eng, com, slots, cs, dev = setup
    # serial references (and the oracle on every certificate)
    ref = {b: eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, ZSEED, b)
           for b in (0, 1000, 2000, 3000)}
    assert ref[0][0].astype(bool).tolist() == nw_ref.verify_certs(cs, com, list(range(cs.ncerts)), ZSEED, 8)
    msg = bytes(cs.msgs[3])
    f = int(cs.cert_first[3])
    votes_pk = [bytes(com.pks[s]) for s in cs.signer[f:f + 27]]
    votes_sig = [bytes(s) for s in cs.sigs[f:f + 27]]
    fresh_seed = [bytes([i + 1]) * 32 for i in range(27)]
    fpk, fsig = eng.sign_many(fresh_seed, [msg] * 27)        # keys outside the cache
    want_uncached = eng.verify_batch([msg] * 27, fpk, fsig, ZSEED, 9)
    errors = []

    def dev_worker(base, reps):
        try:
            st = torch.cuda.Stream(device=dev)
            d = _dev_inputs(cs, slots, dev)
            torch.cuda.synchronize()
            with torch.cuda.stream(st):
                for _ in range(reps):
                    ok, flags, stake = _run_dev(eng, cs, d, dev, st, base)
                    st.synchronize()
                    r = ref[base]
                    if not ((ok.cpu().numpy() == r[0]).all() and ((flags.cpu().numpy() & 8 != 0) == r[1]).all()
                            and (stake.cpu().numpy() == r[2].astype(np.int64)).all()):
                        errors.append(("dev", base))
        except Exception as e:   # pragma: no cover - reported below
            errors.append(("dev-exc", repr(e)))

    def host_worker(base, reps):
        try:
            for _ in range(reps):
                r = eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, ZSEED, base)
                if not all((a == b).all() for a, b in zip(r, ref[base])):
                    errors.append(("host", base))
        except Exception as e:   # pragma: no cover
            errors.append(("host-exc", repr(e)))

    def generic_worker(reps):
        try:
            for _ in range(reps):
                if eng.verify_batch([msg] * 27, votes_pk, votes_sig, ZSEED, 3) != \
                        nw_ref.crypto_verify_batch(msg, list(zip(votes_pk, votes_sig)), ZSEED, 3):
                    errors.append(("cached-batch",))
                if eng.verify_batch([msg] * 27, fpk, fsig, ZSEED, 9) != want_uncached:
                    errors.append(("uncached-batch",))
                if eng.verify_strict_many([msg] * 27, fpk, fsig) != [True] * 27:
                    errors.append(("uncached-strict",))
        except Exception as e:   # pragma: no cover
            errors.append(("generic-exc", repr(e)))

    ths = [threading.Thread(target=dev_worker, args=(0, 6)), threading.Thread(target=dev_worker, args=(1000, 6)),
           threading.Thread(target=host_worker, args=(2000, 6)), threading.Thread(target=host_worker, args=(3000, 6)),
           threading.Thread(target=generic_worker, args=(4,))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert want_uncached
    assert not errors, errors[:5]
    assert eng.committee_size() == 40


def test_batches_in_flight_on_three_streams(setup):
    import torch
    eng, com, slots, cs, dev = setup
    d = _dev_inputs(cs, slots, dev)
    sts = [torch.cuda.Stream(device=dev) for _ in range(3)]
    torch.cuda.synchronize()
    bases = [0, 1000, 2000, 3000, 0, 1000, 2000, 3000, 0]
    outs = []
    for i, base in enumerate(bases):          # no synchronization between the calls
        st = sts[i % 3]
        with torch.cuda.stream(st):
            status = torch.full((1,), 99, dtype=torch.int32, device=dev)
            outs.append((base, status) + _run_dev(eng, cs, d, dev, st, base, status=status))
    torch.cuda.synchronize()
    first_flags = {}
    for base, status, ok, flags, stake in outs:
        r = eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, ZSEED, base)
        assert int(status.item()) == 0
        assert (ok.cpu().numpy() == r[0]).all()
        fl = flags.cpu().numpy()
        assert ((fl & 8 != 0) == r[1]).all()
        assert (stake.cpu().numpy() == r[2].astype(np.int64)).all()
        assert (fl == first_flags.setdefault(base, fl)).all()   # every flag bit, run to run


def test_dev_bad_slot_and_range_are_arg_errors(setup):
    import torch
    from narwhal_amd import _lib
    eng, com, slots, cs, dev = setup
    st = torch.cuda.current_stream()
    d = _dev_inputs(cs, slots, dev)
    d["signer"][17] = 10_000                      # outside the 40-key cache
    with pytest.raises(_lib.DeviceError, match="rc=2"):
        _run_dev(eng, cs, d, dev, st, 0)
    status = torch.full((1,), 99, dtype=torch.int32, device=dev)
    ok, flags, stake = _run_dev(eng, cs, d, dev, st, 0, status=status)
    torch.cuda.synchronize()
    assert int(status.item()) == 2                # NW_ERR_ARG, no fault
    assert int(ok[0].item()) == 0 and int(flags[17].item()) & 8 == 0
    # a certificate whose vote range runs past nsigs
    d2 = _dev_inputs(cs, slots, dev)
    d2["n"][cs.ncerts - 1] = 10_000
    with pytest.raises(_lib.DeviceError, match="rc=2"):
        _run_dev(eng, cs, d2, dev, st, 0)
    status.fill_(99)
    ok, flags, stake = _run_dev(eng, cs, d2, dev, st, 0, status=status)
    torch.cuda.synchronize()
    assert int(status.item()) == 2 and int(ok[cs.ncerts - 1].item()) == 0
    # a good call right after still works
    ok, flags, stake = _run_dev(eng, cs, _dev_inputs(cs, slots, dev), dev, st, 0)
    torch.cuda.synchronize()
    r = eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, ZSEED, 0)
    assert (ok.cpu().numpy() == r[0]).all()


def test_null_zseed_rejected(setup):
    from narwhal_amd import _lib
    eng, com, slots, cs, dev = setup
    L = _lib.LIB
    h = eng.handle
    m = (ctypes.c_char_p * 1)(b"x" * 32)
    ln = (ctypes.c_size_t * 1)(32)
    pk = bytes(com.pks[0])
    sg = bytes(cs.sigs[0])
    assert L.nw_verify_batch(h, m, ln, pk, sg, 1, None, 0) == _lib.NW_ERR_ARG
    cert = (_lib.NwCert * 1)(_lib.NwCert(0, 1))
    sl = (ctypes.c_uint32 * 1)(int(slots[cs.signer[0]]))
    out = (ctypes.c_uint8 * 4)()
    assert L.nw_verify_certs(h, cert, 1, sg, sl, bytes(cs.msgs[0]), None, 0, out, None, None) == _lib.NW_ERR_ARG
    first = (ctypes.c_uint32 * 1)(0)
    cnt = (ctypes.c_uint32 * 1)(1)
    assert L.nw_verify_batches(h, 1, first, cnt, m, ln, sl, sg, None, 0, out, None) == _lib.NW_ERR_ARG
    assert L.nw_verify_batches_pk(h, 1, cnt, m, ln, pk, sg, None, 0, out) == _lib.NW_ERR_ARG
    assert L.nw_verify_certs_dev(h, 0, None, None, 0, None, None, None, None, 0, None, None, None, None,
                                 None) == _lib.NW_ERR_ARG


def test_dev_call_before_any_committee_load(setup):
    """A fixed-window context with an empty key cache: nw_verify_certs_dev is NW_ERR_ARG on the host
    (every slot is out of range and there is no table to clamp to), synchronous and asynchronous
    forms alike, and never reaches the GPU."""
    import torch
    from narwhal_amd import _lib
    _, com, slots, cs, dev = setup
    empty = _lib.Engine(device=0, key_window=16)
    try:
        assert empty.committee_size() == 0
        st = torch.cuda.current_stream()
        d = _dev_inputs(cs, slots, dev)
        status = torch.full((1,), 99, dtype=torch.int32, device=dev)
        for s in (None, status):
            with pytest.raises(_lib.DeviceError, match="rc=2"):
                _run_dev(empty, cs, d, dev, st, 0, status=s)
        torch.cuda.synchronize()
    finally:
        empty.close()


def test_committee_reload_while_dev_work_in_flight(setup):
    """nw_committee_load of an already-cached committee with unchanged stakes changes nothing and
    does not drain in-flight _dev calls; a changed stake is applied after them.  Verdicts of the
    in-flight calls are unaffected."""
    import torch
    eng, com, slots, cs, dev = setup
    st = torch.cuda.Stream(device=dev)
    d = _dev_inputs(cs, slots, dev)
    want = eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, ZSEED, 0)
    outs = []
    with torch.cuda.stream(st):
        for _ in range(4):
            outs.append(_run_dev(eng, cs, d, dev, st, 0))
    again = eng.committee_load_np(com.pks, com.stake)            # unchanged: no refresh
    assert (again == slots).all()
    doubled = eng.committee_load_np(com.pks, com.stake * 2)      # changed: drains, then applies
    assert (doubled == slots).all()
    torch.cuda.synchronize()
    for ok, flags, stake in outs:
        assert (ok.cpu().numpy() == want[0]).all()
    r2 = eng.verify_certs_np(cs.cert_first, cs.cert_n, cs.sigs, slots[cs.signer], cs.msgs, ZSEED, 0)
    assert (r2[2] == 2 * want[2]).all()
    eng.committee_load_np(com.pks, com.stake)                     # restore for the other tests
