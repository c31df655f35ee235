"""The worker's batch digesting with batched, asynchronous GPU submissions.

The reference ``Processor`` (worker/src/processor.rs:30-97) takes one serialized batch at a time
from its channel, hashes it (``Sha512::digest(&batch)[..32]``, :65), optionally runs the simulated
signature load (:67-81), stores the batch under its digest (:84) and sends
``WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, id)`` to the primary (:87-96).

One SHA-512 of one 508,052-B batch is a single chain of 3,970 compressions: on the GPU that chain
runs at the lone-chain rate (~12-15 ms), ~40x slower than one host core, whatever else the GPU is
doing.  What the GPU adds is concurrency: up to a thousand such chains run side by side at the same
per-chain rate.  So the drop-in for :65 is not one ``nw_sha512`` per batch but one
``nw_sha512_many_async`` submission per WINDOW of batches:

* ``DigestBatcher.push(batch)`` appends a batch to the open window; a full window (``window``
  batches or ``max_bytes``) is submitted at once.  ``flush()`` submits a partial window (the Rust
  loop calls it when ``try_recv`` finds the channel empty).
* While up to ``depth`` windows are in flight, the loop keeps receiving batches.
* ``ready()`` / ``drain()`` deliver each finished batch's ``(digest, batch)`` in ARRIVAL order: a
  window is delivered only after every earlier window, exactly like the serial loop's order.

``Processor`` mirrors the reference object on top of it: store + the serialized
``WorkerPrimaryMessage`` in arrival order, and, when given a ``VerifyLoad``, the simulated signature
verification of :67-81 on every batch.

The simulated load (``VerifyLoad``).  Each of a worker's TWO Processors (own batches,
worker/src/worker.rs:182; other workers' batches, :228) makes 100,000 fresh keypairs at spawn and
signs the 8-byte LE messages 0..99,999 (processor.rs:46-58); per batch it verifies the first
``min(100,000, #tx)`` of them as 64 ``verify_batch`` chunks and unwraps every verdict (:67-81).
A worker process therefore holds 200,000 distinct keys.  The drop-in: the worker's engine is
created in committee mode with the two Processors' keys declared up front (``worker_engine``:
``max_keys`` = 200,000), so the first Processor's load sizes the comb window for all of them (W9 on
an idle MI355X: 190 GB of tables) and the second appends without a growth copy.  The worker loads
no committee (it verifies no committee signature).  Each batch's 64 chunks are ONE
``nw_verify_batches`` call on the cached comb tables.  Host logic only: every digest and verdict
comes from libnwcrypto; there is no CPU hashing or verification in this module.
"""
from __future__ import annotations

import os
import struct
import warnings
from collections import deque
from typing import Deque, Iterable, Iterator, List, MutableMapping, Optional, Tuple

from . import _lib

OUR_BATCH, OTHERS_BATCH = 0, 1   # WorkerPrimaryMessage variant indices (primary/src/primary.rs:51-56)
SIM_KEYS = 100_000                # simulated-load keypairs per Processor (worker/src/processor.rs:47)
PROCESSORS_PER_WORKER = 2         # own batches (worker/src/worker.rs:182) + others' batches (:228)
SIM_CHUNKS = 64                   # verify_batch chunks per batch (processor.rs:75)
WORKER_MSG_BATCH = 0              # WorkerMessage::Batch variant index (worker/src/worker.rs:37-40)


class VerificationPanic(RuntimeError):
    """The reference ``.unwrap()``s every chunk verdict (processor.rs:78): a failing chunk panics
    the Processor task."""


def worker_engine(device: int = -1, processors: int = PROCESSORS_PER_WORKER, keys: int = SIM_KEYS):
    """The worker process's engine: committee mode (key_window -1) with every
    simulated-load key declared through ``max_keys``, so both Processors' loads are cached on one
    comb window and one allocation."""
    return _lib.Engine(device=device, max_keys=processors * keys, key_window=-1)


def batch_tx_count(batch) -> int:
    """Transactions in a serialized ``WorkerMessage`` (bincode 1.3: u32 LE variant; ``Batch`` =
    u64 LE count, then each transaction as u64 LE length + bytes).  Returns -1 for a well-formed
    ``BatchRequest(Vec<Digest>, PublicKey)`` (worker/src/worker.rs:37-40: u64 LE count, that many
    32-byte digests, then the key as its base64 string, u64 LE length + bytes, crypto/src/lib.rs:94-112;
    the reference's ``if let WorkerMessage::Batch`` does not verify it).  A malformed message of
    either variant raises ValueError where the reference's ``deserialize(..).unwrap()`` panics
    (processor.rs:68)."""
    mv = memoryview(batch).cast("B")
    if len(mv) < 4:
        raise ValueError("WorkerMessage: truncated variant")
    (variant,) = struct.unpack_from("<I", mv, 0)
    if variant != WORKER_MSG_BATCH:
        if variant == 1:
            _check_batch_request(mv)
            return -1
        raise ValueError("WorkerMessage: unknown variant %d" % variant)
    if len(mv) < 12:
        raise ValueError("WorkerMessage::Batch: truncated length")
    (n,) = struct.unpack_from("<Q", mv, 4)
    pos = 12
    for _ in range(n):
        if pos + 8 > len(mv):
            raise ValueError("WorkerMessage::Batch: truncated transaction")
        (ln,) = struct.unpack_from("<Q", mv, pos)
        pos += 8 + ln
        if pos > len(mv):
            raise ValueError("WorkerMessage::Batch: truncated transaction")
    return n


def _check_batch_request(mv) -> None:
    """bincode ``WorkerMessage::BatchRequest(Vec<Digest>, PublicKey)`` after its variant word."""
    from .primary import _b64_decode
    if len(mv) < 12:
        raise ValueError("WorkerMessage::BatchRequest: truncated digest count")
    (n,) = struct.unpack_from("<Q", mv, 4)
    pos = 12 + 32 * n
    if pos + 8 > len(mv):
        raise ValueError("WorkerMessage::BatchRequest: truncated digests or key length")
    (ln,) = struct.unpack_from("<Q", mv, pos)
    if pos + 8 + ln > len(mv):
        raise ValueError("WorkerMessage::BatchRequest: truncated public key")
    raw = _b64_decode(bytes(mv[pos + 8:pos + 8 + ln]))
    if raw is None or len(raw) < 32:
        raise ValueError("WorkerMessage::BatchRequest: bad base64 public key")


def sim_chunks(count: int):
    """processor.rs:76-77: chunk c covers [count*c/64, min(count, count*(c+1)/64))."""
    import numpy as np
    c = np.arange(SIM_CHUNKS, dtype=np.uint64)
    first = (count * c) // SIM_CHUNKS
    end = np.minimum(count, (count * (c + 1)) // SIM_CHUNKS)
    return first.astype(np.uint32), (end - first).astype(np.uint32)


class VerifyLoad:
    """One Processor's simulated signature load (worker/src/processor.rs:46-58 at spawn, :67-81
    per batch) on the GPU.

    At construction: ``keys`` keypairs from fresh seeds (OsRng in the reference; ``seed`` makes
    them reproducible for tests), signatures over the 8-byte LE messages 0..keys-1 (``nw_sign_many``),
    and one ``nw_committee_load`` of the public keys (their cache slots).  ``verify(batch)`` runs the
    64 chunks of one batch as one ``nw_verify_batches`` call with fresh coefficients and raises
    ``VerificationPanic`` when a chunk fails, as the reference's unwrap panics."""

    def __init__(self, engine, keys: int = SIM_KEYS, seed=None):
        import numpy as np
        self.engine = engine
        self.keys = keys
        rng = np.random.default_rng(seed) if seed is not None else None
        seeds = (rng.integers(0, 256, (keys, 32), dtype=np.uint8) if rng is not None
                 else np.frombuffer(os.urandom(32 * keys), np.uint8).reshape(keys, 32))
        self.msgs = np.arange(keys, dtype="<u8").view(np.uint8).reshape(keys, 8)   # i.to_le_bytes()
        self.pks, self.sigs = engine.sign_many_np(seeds, self.msgs)
        self.slots = engine.committee_load_np(self.pks)
        self.verified = 0

    def chunk_verdicts(self, count: int, zseed: bytes = None, batch_base: int = 0):
        """batch_ok[64] of the first ``count`` signatures split as processor.rs:75-79 does."""
        first, n = sim_chunks(count)
        zseed = os.urandom(32) if zseed is None else zseed
        batch_ok, _ = self.engine.verify_batches_np(first, n, self.msgs[:count], self.slots[:count],
                                                    self.sigs[:count], zseed, batch_base)
        return batch_ok

    def verify(self, batch, zseed: bytes = None) -> int:
        """The per-batch load of processor.rs:67-81; returns the number of signatures verified."""
        ntx = batch_tx_count(batch)
        if ntx < 0:
            return 0
        if ntx > self.keys:
            warnings.warn("Batch size maximum for signature verification surpassed! %d" % ntx)
        count = min(self.keys, ntx)
        ok = self.chunk_verdicts(count, zseed)
        if not ok.all():
            raise VerificationPanic("verify_batch chunk(s) %s failed" % [i for i, v in enumerate(ok.tolist()) if not v])
        self.verified += count
        return count


def serialize_worker_primary_message(digest32: bytes, worker_id: int, own_digest: bool) -> bytes:
    """bincode 1.3 of WorkerPrimaryMessage::{OurBatch, OthersBatch}(Digest, WorkerId): u32 LE variant
    index, the 32 digest bytes (a fixed array: no length prefix), u32 LE worker id."""
    if len(digest32) != 32:
        raise ValueError("Digest is 32 bytes")
    return struct.pack("<I", OUR_BATCH if own_digest else OTHERS_BATCH) + bytes(digest32) + struct.pack("<I", worker_id)


class DigestBatcher:
    """Windows of batches -> one asynchronous GPU submission each; results in arrival order."""

    # max_bytes: a window is cut into several submissions only above 1 GiB of batches.  C4's
    # per-GPU window (1,250 x 508,052 B = 635 MB) as ONE submission: 41.2-41.7 k batches/s against
    # 21.0-22.0 k when a 256 MiB cap cut it into three jobs (depth 2 or 4: concurrent jobs of one
    # context do not overlap their digests, profiles/r06/worker_window_r06.txt).  The price is one
    # pinned staging buffer of the window's size per workspace in flight.
    def __init__(self, engine=None, window: int = 64, depth: int = 2, max_bytes: int = 1 << 30):
        if window < 1 or depth < 1:
            raise ValueError("window and depth must be >= 1")
        self.engine = engine or _lib.default_engine()
        self.window, self.depth, self.max_bytes = window, depth, max_bytes
        self._open: List = []
        self._open_bytes = 0
        self._inflight: Deque[Tuple[List, "_lib.DigestJob"]] = deque()
        self._done: Deque[Tuple[bytes, object]] = deque()
        self.submissions = 0

    def push(self, batch) -> None:
        """Accept one serialized batch (bytes-like, kept referenced until delivered)."""
        self._open.append(batch)
        self._open_bytes += len(batch)
        if len(self._open) >= self.window or self._open_bytes >= self.max_bytes:
            self.flush()

    def flush(self) -> None:
        """Submit the open window, however small (no-op when empty)."""
        if not self._open:
            return
        while len(self._inflight) >= self.depth:   # bounded in-flight work: retire the oldest first
            self._retire_oldest()
        batches, self._open, self._open_bytes = self._open, [], 0
        self._inflight.append((batches, self.engine.sha512_many_submit(batches)))
        self.submissions += 1

    def _retire_oldest(self) -> None:
        batches, job = self._inflight.popleft()
        for b, d in zip(batches, job.wait()):
            self._done.append((d, b))

    def ready(self) -> List[Tuple[bytes, object]]:
        """(64-byte digest, batch) of every batch whose window and all earlier windows are done;
        never blocks."""
        while self._inflight and self._inflight[0][1].done():
            self._retire_oldest()
        out = list(self._done)
        self._done.clear()
        return out

    def drain(self) -> List[Tuple[bytes, object]]:
        """Submit the open window and wait for everything pushed so far (arrival order)."""
        self.flush()
        while self._inflight:
            self._retire_oldest()
        out = list(self._done)
        self._done.clear()
        return out

    def pending(self) -> int:
        return len(self._open) + sum(len(b) for b, _ in self._inflight) + len(self._done)

    def pipeline(self, batches: Iterable) -> Iterator[Tuple[bytes, object]]:
        """The Processor loop over an iterable channel: push every batch, deliver whatever is ready
        between arrivals, drain at the end.  Yields (digest, batch) in arrival order."""
        for b in batches:
            self.push(b)
            yield from self.ready()
        yield from self.drain()


class Processor:
    """worker/src/processor.rs ``Processor`` (digest, store, deliver) over a ``DigestBatcher``.

    ``run(batches)`` yields the serialized ``WorkerPrimaryMessage`` the reference sends on
    ``tx_digest`` for each batch, in arrival order, after storing ``store[digest32] = batch``.
    With ``verify`` (a ``VerifyLoad``: ``enable_verification``, processor.rs:43-58) every batch also
    runs the simulated signature load when it arrives; a failing chunk raises ``VerificationPanic``
    before that batch is stored or delivered, as the reference's unwrap panics the task."""

    def __init__(self, worker_id: int, own_digest: bool, store: Optional[MutableMapping] = None, engine=None,
                 window: int = 64, depth: int = 2, verify: Optional[VerifyLoad] = None):
        self.id = worker_id
        self.own_digest = own_digest
        self.store = store if store is not None else {}
        self.batcher = DigestBatcher(engine, window=window, depth=depth)
        self.verify = verify

    def _deliver(self, items) -> Iterator[bytes]:
        for digest64, batch in items:
            d = digest64[:32]
            self.store[d] = bytes(batch)
            yield serialize_worker_primary_message(d, self.id, self.own_digest)

    def run(self, batches: Iterable) -> Iterator[bytes]:
        for b in batches:
            if self.verify is not None:
                try:
                    self.verify.verify(b)
                except VerificationPanic:
                    # the reference's task had stored and delivered every earlier batch before it
                    # panicked on this one: deliver what is in flight, then fail
                    yield from self._deliver(self.batcher.drain())
                    raise
            self.batcher.push(b)
            yield from self._deliver(self.batcher.ready())
        yield from self._deliver(self.batcher.drain())
