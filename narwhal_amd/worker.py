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
``WorkerPrimaryMessage`` in arrival order.  The simulated verify load (:67-81) is the separate
``nw_verify_batches`` / ``nw_verify_batches_pk`` path.  Host logic only: every
digest comes from libnwcrypto; there is no CPU hashing in this module.
"""
from __future__ import annotations

import struct
from collections import deque
from typing import Deque, Iterable, Iterator, List, MutableMapping, Optional, Tuple

from . import _lib

OUR_BATCH, OTHERS_BATCH = 0, 1   # WorkerPrimaryMessage variant indices (primary/src/primary.rs:51-56)


def serialize_worker_primary_message(digest32: bytes, worker_id: int, own_digest: bool) -> bytes:
    """bincode 1.3 of WorkerPrimaryMessage::{OurBatch, OthersBatch}(Digest, WorkerId): u32 LE variant
    index, the 32 digest bytes (a fixed array: no length prefix), u32 LE worker id."""
    if len(digest32) != 32:
        raise ValueError("Digest is 32 bytes")
    return struct.pack("<I", OUR_BATCH if own_digest else OTHERS_BATCH) + bytes(digest32) + struct.pack("<I", worker_id)


class DigestBatcher:
    """Windows of batches -> one asynchronous GPU submission each; results in arrival order."""

    def __init__(self, engine=None, window: int = 64, depth: int = 2, max_bytes: int = 256 << 20):
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
    ``tx_digest`` for each batch, in arrival order, after storing ``store[digest32] = batch``."""

    def __init__(self, worker_id: int, own_digest: bool, store: Optional[MutableMapping] = None, engine=None,
                 window: int = 64, depth: int = 2):
        self.id = worker_id
        self.own_digest = own_digest
        self.store = store if store is not None else {}
        self.batcher = DigestBatcher(engine, window=window, depth=depth)

    def _deliver(self, items) -> Iterator[bytes]:
        for digest64, batch in items:
            d = digest64[:32]
            self.store[d] = bytes(batch)
            yield serialize_worker_primary_message(d, self.id, self.own_digest)

    def run(self, batches: Iterable) -> Iterator[bytes]:
        for b in batches:
            self.batcher.push(b)
            yield from self._deliver(self.batcher.ready())
        yield from self._deliver(self.batcher.drain())
