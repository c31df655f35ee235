"""GPU: the worker's batched asynchronous digest path (nw_sha512_many_async via
narwhal_amd.worker) against hashlib and the reference's own Processor test.

* worker/src/tests/processor_tests.rs:9-48 (hash_and_store): the golden serialized batch gives
  WorkerPrimaryMessage::OurBatch(digest, 0) and is stored under that digest;
* 150 batches in arrival order through windows of 16 with 3 in flight: C4-shape bincode batches
  (508,052 B, node/src/benchmark_client.rs tx layout), small and empty batches, unaligned host
  buffers, partial windows flushed mid-stream;
* C4's 635 MB window as one submission (default byte cap), then a second window;
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


def test_c4_window_is_one_submission(engine):
    """C4's per-GPU window (1,250 x 508,052 B = 635 MB, worker/src/processor.rs:63-65 for each
    batch) goes out as ONE nw_sha512_many_async job under the default byte cap, every digest equal
    to hashlib's; a second window follows through the same batcher (pinned buffer reuse)."""
    from narwhal_amd import worker, workload
    host = workload.worker_batches_np(1250)
    rows = [host[i].copy() for i in range(1250)]
    for k in range(0, 1250, 97):                    # distinct contents along the window
        rows[k][100:108] = np.frombuffer(struct.pack("<Q", k + 1), np.uint8)
    b = worker.DigestBatcher(engine, window=1250, depth=2)
    got = []
    for x in rows:
        b.push(x)
        got += b.ready()
    assert b.submissions == 1
    tail = [r.copy() for r in rows[:300]]
    for x in tail:
        b.push(x)
    got += b.drain()
    assert b.submissions == 2
    assert len(got) == 1550
    for (d, x), want in zip(got, rows + tail):
        assert x is want
        assert d == hashlib.sha512(want.tobytes()).digest()


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


def test_worker_spawn_sequence_two_processors_cached():
    """INTEGRATION.md §3, the worker process exactly as documented:
    * the engine is created in committee mode with both Processors' simulation keys declared
      (``worker_engine``: max_keys 200,000); Worker::spawn loads NO committee;
    * Processor::spawn for our batches (worker/src/worker.rs:182), then for others' batches (:228):
      each makes 100,000 keypairs, signs the LE messages 0..99,999 and loads its keys
      (processor.rs:46-58); the second load must not hit NW_ERR_NOMEM;
    * per batch: min(100,000, #tx) signatures in 64 verify_batch chunks (processor.rs:67-81) as ONE
      nw_verify_batches call on the cached combs.  Chunk verdicts against the C restatement of
      dalek (oracle/nw_ref.c) with the same coefficients, including chunks with a corrupted
      signature; a 100,001-transaction batch verifies the full 100,000; ``Processor`` with the load
      delivers every batch's digest."""
    import nw_ref
    from narwhal_amd import workload, worker as w
    eng = w.worker_engine(device=0)
    try:
        own = w.VerifyLoad(eng, seed=5)       # Processor::spawn(.., own_digest = true, ..)
        others = w.VerifyLoad(eng, seed=6)    # Processor::spawn(.., own_digest = false, ..)
        assert eng.committee_size() == 2 * w.SIM_KEYS
        assert eng.key_window() in (8, 9), eng.key_window()
        print("worker engine: window W%d for %d keys" % (eng.key_window(), eng.committee_size()))
        assert not np.array_equal(own.pks[:8], others.pks[:8])

        def oracle_chunks(load, count, zseed, base, only=None):
            first, n = w.sim_chunks(count)
            want = []
            for c in range(64):
                if only is not None and c not in only:
                    want.append(None)
                    continue
                f, k = int(first[c]), int(n[c])
                want.append(nw_ref.verify_batch_msgs([bytes(m) for m in load.msgs[f:f + k]],
                                                     [bytes(p) for p in load.pks[f:f + k]],
                                                     [bytes(s) for s in load.sigs[f:f + k]], zseed, base + c))
            return want

        zseed = bytes(range(7, 39))
        for load in (own, others):                       # a C4-shape batch: 977 transactions
            got = load.chunk_verdicts(977, zseed, 0).astype(bool).tolist()
            assert got == oracle_chunks(load, 977, zseed, 0) == [True] * 64
        # corrupted signatures in three chunks of our Processor's load (a bit of R, S + l, another message)
        saved = own.sigs.copy()
        try:
            own.sigs[100, 3] ^= 0x10
            sv = int.from_bytes(bytes(own.sigs[500, 32:]), "little") + (2 ** 252 + 27742317777372353535851937790883648493)
            own.sigs[500, 32:] = np.frombuffer(sv.to_bytes(32, "little"), np.uint8)
            own.sigs[900] = others.sigs[900]
            got = own.chunk_verdicts(977, zseed, 64).astype(bool).tolist()
            want = oracle_chunks(own, 977, zseed, 64)
            assert got == want
            first, n = w.sim_chunks(977)
            hit = sorted({c for i in (100, 500, 900) for c in range(64) if first[c] <= i < first[c] + n[c]})
            assert [c for c in range(64) if not got[c]] == hit and len(hit) == 3
            with pytest.raises(w.VerificationPanic):
                own.verify(workload.worker_batch(977, 512))
        finally:
            own.sigs[:] = saved
        # a batch above the simulation maximum: the first 100,000 signatures (processor.rs:70-73)
        big = workload.worker_batch(w.SIM_KEYS + 1, 9)
        with pytest.warns(UserWarning, match="maximum"):
            assert others.verify(big) == w.SIM_KEYS
        got = others.chunk_verdicts(w.SIM_KEYS, zseed, 1000).astype(bool).tolist()
        assert got == [True] * 64
        want = oracle_chunks(others, w.SIM_KEYS, zseed, 1000, only={0, 31, 63})
        assert [want[0], want[31], want[63]] == [True] * 3
        # the Processor loop with the load enabled: digests as the reference's hash_and_store
        batches = [workload.worker_batch(977, 512, b) for b in range(3)] + [workload.worker_batch(10, 32, 9)]
        p = w.Processor(worker_id=2, own_digest=True, engine=eng, window=2, depth=2, verify=own)
        out = list(p.run(batches))
        assert [m[4:36] for m in out] == [hashlib.sha512(b).digest()[:32] for b in batches]
        assert own.verified == 3 * 977 + 10
    finally:
        eng.close()
