"""CPU: the multi-GPU sharding layer (narwhal_amd/shard.py) with world_size 2 over gloo —
partition balance, and the verdict/stake all-gather reproducing the single-process arrays."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from narwhal_amd import shard


def test_partition_balanced_and_covering():
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        for _ in range(20):
            n = rng.integers(0, 200)
            cert_n = rng.integers(0, 700, size=n)
            r = shard.partition(cert_n, world)
            assert len(r) == world and r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            if n and cert_n.sum():
                loads = [cert_n[c0:c1].sum() for c0, c1 in r]
                assert max(loads) - cert_n.sum() / world <= cert_n.max() + 1


def test_pack_unpack_roundtrip():
    for n in (0, 1, 7, 8, 9, 1000):
        ok = torch.randint(0, 2, (n,), dtype=torch.uint8)
        assert torch.equal(shard.unpack_bits(shard.pack_bits(ok), n), ok)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cert_n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ranges = shard.partition(cert_n, world)
    c0, c1 = ranges[rank]
    idx = torch.arange(c0, c1)
    ok = ((idx * 7 + 3) % 5 != 0).to(torch.uint8)      # deterministic "verdicts" per global index
    stake = (idx * 13) % 101
    gok, gst = shard.allgather_verdicts(ok, stake.to(torch.int64), ranges)
    q.put((rank, gok.numpy().tolist(), gst.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_allgather_verdicts_gloo(world):
    cert_n = np.random.default_rng(1).integers(1, 100, size=123)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cert_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx = np.arange(len(cert_n))
    want_ok = ((idx * 7 + 3) % 5 != 0).astype(int).tolist()
    want_st = ((idx * 13) % 101).tolist()
    for rank, gok, gst in res:
        assert gok == want_ok and gst == want_st, rank


# ----------------------------------------------------------------------------- plumbing with stub engines
class _StubCertEngine:
    """Stands in for _lib.Engine.verify_certs_np: verdict / stake are functions of the GLOBAL
    certificate index (cert_base + local index), so a wrong shard offset shows up."""

    def verify_certs_np(self, cert_first, cert_n, sigs, slots, msgs, zseed, cert_base=0):
        nc = len(cert_n)
        assert sigs.shape[0] == int(np.sum(cert_n)) == slots.shape[0]
        assert nc == 0 or int(cert_first[0]) == 0
        g = np.arange(cert_base, cert_base + nc)
        ok = ((g * 7 + 3) % 5 != 0).astype(np.uint8)
        return ok, np.ones(sigs.shape[0], np.uint8), (np.asarray(cert_n, np.uint64) * 3 + g.astype(np.uint64))


class _StubSplitEngine:
    """Stands in for verify_batch_partial / points_sum_is_identity: a shard's "point" encodes the
    z offset and count it was called with; the sum is the identity iff the shards tile [0, n)."""

    def __init__(self, n, bad_at=None):
        self.n, self.bad_at = n, bad_at

    def verify_batch_partial(self, msgs, pks, sigs, zseed, batch_index, z_offset):
        k = len(sigs)
        assert len(msgs) == len(pks) == k
        pt = (z_offset.to_bytes(8, "little") + k.to_bytes(8, "little")).ljust(160, b"\0")
        bad = self.bad_at is not None and z_offset <= self.bad_at < z_offset + k
        return pt, bad

    def points_sum_is_identity(self, points):
        spans = sorted((int.from_bytes(p[:8], "little"), int.from_bytes(p[8:16], "little")) for p in points)
        pos = 0
        for a, k in spans:
            if a != pos:
                return False
            pos += k
        return pos == self.n


class _Certs:
    def __init__(self, cert_n):
        self.cert_n = np.asarray(cert_n, np.uint32)
        self.cert_first = np.concatenate([[0], np.cumsum(self.cert_n)[:-1]]).astype(np.uint32)
        n = int(self.cert_n.sum())
        self.sigs = np.zeros((n, 64), np.uint8)
        self.signer = np.zeros(n, np.uint32)
        self.msgs = np.zeros((len(cert_n), 32), np.uint8)


def _plumbing_worker(rank, world, port, cert_n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cs = _Certs(cert_n)
    ok, st = shard.verify_sharded(_StubCertEngine(), cs, np.zeros(4, np.uint32), bytes(32), rank, world,
                                  device=torch.device("cpu"))
    n = 6667
    msgs = [b"m"] * n
    v_ok = shard.verify_split_batch(_StubSplitEngine(n), msgs, msgs, msgs, bytes(32), 5, rank, world,
                                    device=torch.device("cpu"))
    v_bad = shard.verify_split_batch(_StubSplitEngine(n, bad_at=6000), msgs, msgs, msgs, bytes(32), 5, rank, world,
                                     device=torch.device("cpu"))
    q.put((rank, ok.numpy().tolist(), st.numpy().tolist(), v_ok, v_bad))
    dist.barrier()
    dist.destroy_process_group()


def test_verify_sharded_and_split_batch_plumbing_gloo():
    world = 2
    cert_n = np.random.default_rng(2).integers(1, 80, size=57)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plumbing_worker, args=(r, world, port, cert_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.arange(len(cert_n))
    want_ok = ((g * 7 + 3) % 5 != 0).astype(int).tolist()
    want_st = (cert_n * 3 + g).tolist()
    for rank, ok, st, v_ok, v_bad in res:
        assert ok == want_ok and st == want_st, rank
        assert v_ok is True and v_bad is False, rank


def _digest_worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64)
    local = ((g[:, None] * 31 + torch.arange(64)[None, :] * 7) % 251).to(torch.uint8)   # [n, 64] per rank
    out = shard.allgather_digests(local)
    q.put((rank, out.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_allgather_digests_gloo():
    """C4's worker digests across ranks: every rank ends with every rank's first 32
    digest bytes per batch, in rank order."""
    world, n = 2, 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_digest_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.arange(world * n)[:, None]
    want = ((g * 31 + np.arange(32)[None, :] * 7) % 251).tolist()
    for rank, got in res:
        assert got == want, rank
