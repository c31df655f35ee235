"""CPU: host logic of the worker's batched digest path (narwhal_amd/worker.py) with a stand-in
engine whose jobs complete on demand; the digests themselves are the GPU's (tests/test_gpu_worker.py).

* bincode of WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, id) as the reference serializes
  it (worker/src/tests/processor_tests.rs:36-44: the expected output of hash_and_store);
* windows: full windows submit at once, flush() submits a partial one, max_bytes cuts a window;
* at most ``depth`` submissions in flight; deliveries in arrival order even when a later window
  completes first.
"""
import hashlib
import json
import os
import struct

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeJob:
    def __init__(self, log, msgs):
        self.msgs = [bytes(m) for m in msgs]
        self.complete = False
        self.log = log

    def done(self):
        return self.complete

    def wait(self):
        self.log.append(("wait", len(self.msgs)))
        self.complete = True
        return [hashlib.sha512(m).digest() for m in self.msgs]


class FakeEngine:
    """Stand-in for _lib.Engine.sha512_many_submit (test scaffolding, not a product path)."""

    def __init__(self):
        self.jobs = []
        self.log = []

    def sha512_many_submit(self, msgs):
        j = FakeJob(self.log, msgs)
        self.jobs.append(j)
        self.log.append(("submit", len(j.msgs)))
        return j


def _import():
    import importlib
    import sys
    sys.modules.pop("narwhal_amd.worker", None)
    # worker.py imports _lib (which loads libnwcrypto.so); the host logic needs only the engine
    # passed in, so the library must be present (it is built by __graft_entry__.build()).
    return importlib.import_module("narwhal_amd.worker")


def test_serialize_matches_reference_layout():
    w = _import()
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        g = json.load(f)["worker_batch"]
    d = bytes.fromhex(g["digest"])
    assert w.serialize_worker_primary_message(d, 0, True) == struct.pack("<I", 0) + d + struct.pack("<I", 0)
    assert w.serialize_worker_primary_message(d, 7, False) == struct.pack("<I", 1) + d + struct.pack("<I", 7)
    with pytest.raises(ValueError):
        w.serialize_worker_primary_message(d[:31], 0, True)


def test_windows_partial_flush_and_order():
    w = _import()
    eng = FakeEngine()
    b = w.DigestBatcher(eng, window=4, depth=2)
    batches = [os.urandom(100 + i) for i in range(10)]
    for x in batches[:4]:
        b.push(x)
    assert eng.log == [("submit", 4)]            # a full window goes out at once
    for x in batches[4:6]:
        b.push(x)
    assert b.ready() == []                       # nothing completed yet
    b.flush()                                    # partial window (the channel ran dry)
    assert eng.log[-1] == ("submit", 2)
    eng.jobs[1].complete = True                  # the later window finishes first ...
    assert b.ready() == []                       # ... but is held behind the earlier one
    eng.jobs[0].complete = True
    got = b.ready()
    assert [x for _, x in got] == batches[:6]
    assert [d for d, _ in got] == [hashlib.sha512(x).digest() for x in batches[:6]]
    for x in batches[6:]:
        b.push(x)
    rest = b.drain()
    assert [x for _, x in rest] == batches[6:] and b.pending() == 0


def test_depth_bounds_inflight_and_max_bytes():
    w = _import()
    eng = FakeEngine()
    b = w.DigestBatcher(eng, window=2, depth=2, max_bytes=1000)
    for i in range(6):
        b.push(bytes([i]) * 10)
    # three full windows: the third submission first retires the oldest (depth 2)
    assert [e for e in eng.log if e[0] == "submit"] == [("submit", 2)] * 3
    assert eng.log.index(("wait", 2)) < len(eng.log) - 1
    b2 = w.DigestBatcher(FakeEngine(), window=100, depth=1, max_bytes=1000)
    b2.push(b"x" * 600)
    assert b2.submissions == 0
    b2.push(b"y" * 600)                          # 1,200 bytes >= max_bytes: submitted
    assert b2.submissions == 1
    assert len(b2.drain()) == 2


def test_processor_store_and_messages():
    w = _import()
    p = w.Processor(worker_id=3, own_digest=False, engine=FakeEngine(), window=3, depth=2)
    batches = [os.urandom(50 * (i + 1)) for i in range(7)]
    out = list(p.run(batches))
    want = [w.serialize_worker_primary_message(hashlib.sha512(x).digest()[:32], 3, False) for x in batches]
    assert out == want
    assert all(p.store[hashlib.sha512(x).digest()[:32]] == x for x in batches)


def test_bad_parameters():
    w = _import()
    with pytest.raises(ValueError):
        w.DigestBatcher(FakeEngine(), window=0)
    with pytest.raises(ValueError):
        w.DigestBatcher(FakeEngine(), depth=0)


# ----------------------------------------------------------------------- simulated verify load (A13)
def test_batch_tx_count_parses_worker_messages():
    """worker/src/processor.rs:68-70: bincode WorkerMessage; Batch -> its transaction count,
    BatchRequest -> not verified, malformed -> error (the reference's unwrap panics)."""
    from narwhal_amd import workload
    w = _import()
    assert w.batch_tx_count(workload.worker_batch(977, 512)) == 977
    assert w.batch_tx_count(workload.worker_batch(0, 512)) == 0
    assert w.batch_tx_count(workload.worker_batch(5, 9)) == 5
    import base64
    key = base64.b64encode(bytes(range(32)))                            # PublicKey: its base64 string
    req = struct.pack("<IQ", 1, 2) + bytes(64) + struct.pack("<Q", len(key)) + key   # BatchRequest(2 digests, origin)
    assert w.batch_tx_count(req) == -1
    assert w.batch_tx_count(struct.pack("<IQ", 1, 0) + struct.pack("<Q", len(key)) + key) == -1
    short = base64.b64encode(bytes(24))                                 # decodes to < 32 bytes
    good = workload.worker_batch(3, 16)
    for bad in (good[:-1], good[:10], b"\x02\0\0\0", b"", req[:-1], req[:40], req[:12],
                struct.pack("<IQ", 1, 0) + struct.pack("<Q", len(short)) + short,
                struct.pack("<IQ", 1, 0) + struct.pack("<Q", 4) + b"!!!!"):
        with pytest.raises(ValueError):
            w.batch_tx_count(bad)


@pytest.mark.parametrize("count", [0, 1, 63, 64, 977, 100_000])
def test_sim_chunks_match_reference_split(count):
    """processor.rs:75-77: chunk c = [count*c/64, min(count, count*(c+1)/64)) in integer arithmetic;
    the chunks tile [0, count) in order."""
    w = _import()
    first, n = w.sim_chunks(count)
    want = [((count * c) // 64, min(count, (count * (c + 1)) // 64)) for c in range(64)]
    assert [(int(f), int(f + k)) for f, k in zip(first, n)] == want
    assert int(n.sum()) == count


class _FakeLoad:
    """Stand-in VerifyLoad: fails on the batches whose index is in ``bad``."""

    def __init__(self, w, bad=()):
        self.w, self.bad, self.seen = w, set(bad), []

    def verify(self, batch):
        w = self.w
        i = len(self.seen)
        self.seen.append(w.batch_tx_count(batch))
        if i in self.bad:
            raise w.VerificationPanic("chunk 0 failed")
        return self.seen[-1]


def test_processor_runs_verify_load_and_delivers_before_panic():
    """Every batch runs the simulated load on arrival; a failing batch raises after every earlier
    batch was stored and delivered, and is itself neither stored nor delivered (the reference's
    task panics at the unwrap, processor.rs:78, before :84)."""
    from narwhal_amd import workload
    w = _import()
    batches = [workload.worker_batch(4, 16, b) for b in range(5)]
    load = _FakeLoad(w)
    p = w.Processor(worker_id=1, own_digest=True, engine=FakeEngine(), window=2, depth=2, verify=load)
    out = list(p.run(batches))
    assert len(out) == 5 and load.seen == [4] * 5
    load = _FakeLoad(w, bad={3})
    p = w.Processor(worker_id=1, own_digest=True, engine=FakeEngine(), window=2, depth=2, verify=load)
    got = []
    with pytest.raises(w.VerificationPanic):
        for m in p.run(batches):
            got.append(m)
    assert len(got) == 3 and len(p.store) == 3
    assert set(p.store) == {hashlib.sha512(b).digest()[:32] for b in batches[:3]}
