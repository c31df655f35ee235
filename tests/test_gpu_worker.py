"""GPU: the worker's batched asynchronous digest path (nw_sha512_many_async via
narwhal_amd.worker) against hashlib and the reference's own Processor test.

* worker/src/tests/processor_tests.rs:9-48 (hash_and_store): the golden serialized batch gives
  WorkerPrimaryMessage::OurBatch(digest, 0) and is stored under that digest;
* 150 batches in arrival order through windows of 16 with 3 in flight: C4-shape bincode batches
  (508,052 B, node/src/benchmark_client.rs tx layout), small and empty batches, unaligned host
  buffers, partial windows flushed mid-stream;
* the raw ABI: a job polls not-done/done, an empty job, jobs waited out of submission order.
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_processor_hash_and_store_reference(engine):
    from narwhal_amd import worker
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        g = json.load(f)["worker_batch"]
    ser = bytes.fromhex(g["serialized"])
    p = worker.Processor(worker_id=0, own_digest=True, engine=engine)
    out = list(p.run([ser]))
    digest = bytes.fromhex(g["digest"])
    assert out == [struct.pack("<I", 0) + digest + struct.pack("<I", 0)]
    assert p.store[digest] == ser


def test_batched_digests_in_arrival_order(engine):
    from narwhal_amd import worker, workload
    rng = np.random.default_rng(5)
    big = workload.worker_batches_np(40)                      # 40 x 508,052 B
    raw = bytes(rng.integers(0, 256, 3_000_000, dtype=np.uint8))
    batches = []
    for i in range(150):
        k = i % 5
        if k == 0:
            batches.append(big[(i // 5) % 40])                   # numpy row (aligned)
        elif k == 1:
            o = 1 + (i % 7)
            batches.append(memoryview(raw)[o:o + 508_052 + i])  # unaligned host buffer
        elif k == 2:
            batches.append(bytes(rng.integers(0, 256, int(rng.integers(0, 400)), dtype=np.uint8)))
        elif k == 3:
            batches.append(b"")
        else:
            batches.append(bytes(rng.integers(0, 256, 128 * int(rng.integers(1, 40)) - 17, dtype=np.uint8)))
    b = worker.DigestBatcher(engine, window=16, depth=3)
    got = []
    for i, x in enumerate(batches):
        b.push(x)
        if i % 37 == 36:
            b.flush()                                          # partial windows mid-stream
        got += b.ready()
    got += b.drain()
    assert len(got) == len(batches)
    for (d, x), want in zip(got, batches):
        assert x is want
        assert d == hashlib.sha512(bytes(want)).digest()
    assert b.submissions >= len(batches) // 16


def test_async_abi_poll_and_out_of_order_wait(engine):
    import time
    from narwhal_amd import workload
    big = workload.worker_batches_np(64)
    j1 = engine.sha512_many_submit([big[i] for i in range(64)])
    j2 = engine.sha512_many_submit([b"abc", b"", bytes(200)])
    j0 = engine.sha512_many_submit([])
    assert j0.done() and j0.wait() == []
    t0 = time.time()
    while not j2.done():
        assert time.time() - t0 < 30
        time.sleep(0.001)
    assert j2.wait() == [hashlib.sha512(m).digest() for m in (b"abc", b"", bytes(200))]
    d1 = j1.wait()
    assert d1 == [hashlib.sha512(big[i].tobytes()).digest() for i in range(64)]


def test_async_window_above_parallel_staging_threshold(engine):
    """A window of ~41 MB (above the 32 MiB threshold where nw_sha512_many_async packs with helper
    threads, chunk DMAs issued in order as chunks complete): odd lengths, unaligned sources and
    empty messages at chunk edges all hash like hashlib."""
    rng = np.random.default_rng(11)
    raw = bytes(rng.integers(0, 256, 600_000, dtype=np.uint8))
    msgs = []
    for i in range(90):
        if i % 9 == 4:
            msgs.append(b"")
        elif i % 3 == 0:
            o = 1 + i % 13
            msgs.append(memoryview(raw)[o:o + 508_052 + 3 * i])
        else:
            msgs.append(bytes(rng.integers(0, 256, 508_000 + 17 * i, dtype=np.uint8)))
    assert sum(len(m) for m in msgs) > 32 << 20
    got = engine.sha512_many_submit(msgs).wait()
    assert got == [hashlib.sha512(bytes(m)).digest() for m in msgs]
