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
