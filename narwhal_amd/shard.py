"""Multi-GPU sharding of certificate verification.

Certificates are independent units (``Certificate::verify``, primary/src/messages.rs:189-215), so
a node's batch is split into contiguous certificate ranges balanced by vote count, one per GPU
(one process per GPU).  Coefficient streams are keyed by the *global* certificate index
(NW-Z v1 nonce), so a shard needs nothing from the others to reproduce the single-GPU verdicts.
The only exchanges are the RCCL all-gathers of the per-shard verdict bitmaps and stake tallies
(a few KB: latency-bound, one xGMI hop) and, at C4, of the ranks' worker-batch digests (32 B per batch).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def partition(cert_n: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [c0, c1) certificate ranges, one per rank, balanced by total votes."""
    cert_n = np.asarray(cert_n, dtype=np.int64)
    nc = cert_n.shape[0]
    if world <= 1:
        return [(0, nc)]
    cum = np.concatenate([[0], np.cumsum(cert_n)])
    total = int(cum[-1])
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        c = int(np.searchsorted(cum, target, side="left"))
        c = max(bounds[-1], min(c, nc))
        bounds.append(c)
    bounds.append(nc)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def pack_bits(ok):
    """uint8 0/1 tensor [n] -> packed little-endian bit tensor [ceil(n/8)] (torch)."""
    import torch
    n = ok.shape[0]
    nb = (n + 7) // 8
    pad = nb * 8 - n
    bits = torch.nn.functional.pad(ok.to(torch.uint8), (0, pad)).view(nb, 8).to(torch.int32)
    w = (2 ** torch.arange(8, device=ok.device, dtype=torch.int32))
    return (bits * w).sum(dim=1).to(torch.uint8)


def unpack_bits(packed, n: int):
    import torch
    w = (2 ** torch.arange(8, device=packed.device, dtype=torch.int32))
    bits = (packed.to(torch.int32).unsqueeze(1) & w) != 0
    return bits.reshape(-1)[:n].to(torch.uint8)


def allgather_verdicts(ok_local, stake_local, ranges: List[Tuple[int, int]], group=None):
    """All-gather per-shard verdicts (bit-packed) and accepted stake into global [ncerts] tensors.

    ``ok_local``: uint8 [c1 - c0]; ``stake_local``: int64 [c1 - c0] (this rank's range).  One
    collective per call: each rank contributes [bitmap | stake as bytes] in a single uint8 buffer,
    so the exchange is one latency-bound all_gather (RCCL over xGMI on GPU tensors, gloo on CPU
    tensors for the tests)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    maxc = max(c1 - c0 for c0, c1 in ranges)
    maxb = (maxc + 63) // 64 * 8           # bitmap bytes, padded so the stake words stay 8-B aligned
    dev = ok_local.device
    buf = torch.zeros(maxb + 8 * maxc, dtype=torch.uint8, device=dev)
    pb = pack_bits(ok_local)
    buf[:pb.shape[0]] = pb
    n = stake_local.shape[0]
    if n:
        buf[maxb:maxb + 8 * n] = stake_local.to(torch.int64).contiguous().view(torch.uint8)
    gathered = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(gathered, buf, group=group)
    oks, stakes = [], []
    for r, (c0, c1) in enumerate(ranges):
        g = gathered[r]
        oks.append(unpack_bits(g[:maxb], c1 - c0))
        stakes.append(g[maxb:maxb + 8 * (c1 - c0)].view(torch.int64))
    return torch.cat(oks), torch.cat(stakes)


def allgather_digests(digests_local, group=None):
    """All-gather the worker-batch digests of every rank ("worker digests are
    all-gathered the same way, 32 B per batch").  ``digests_local``: uint8 [n, >= 32] on this rank (the
    64-byte SHA-512 outputs; the reference keeps the first 32, worker/src/processor.rs:65).  Every rank
    contributes the same n (the per-rank batch share); returns uint8 [world * n, 32] in rank order.
    One latency-bound collective (RCCL over xGMI on GPU tensors, gloo on CPU tensors)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    local = digests_local[:, :32].contiguous()
    out = torch.empty((world * local.shape[0], 32), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out


def shard_inputs(cs, slots, rank: int, world: int, cert_base: int = 0):
    """This rank's share of ``cs`` (narwhal_amd.workload.Certificates with contiguous vote ranges):
    a dict with ``ranges`` (every rank's [c0, c1)), ``cert_base`` = cert_base + c0 (the GLOBAL index of
    its first certificate: the NW-Z coefficient nonce, so the shard's verdicts equal the one-GPU
    verdicts of a call with batch index ``cert_base``),
    and its rebased arrays ``first``, ``n``, ``sigs``, ``signer_slots``, ``msgs``."""
    ranges = partition(cs.cert_n, world)
    c0, c1 = ranges[rank]
    f0 = int(cs.cert_first[c0]) if c1 > c0 else 0
    f1 = int(cs.cert_first[c1 - 1] + cs.cert_n[c1 - 1]) if c1 > c0 else 0
    return {"ranges": ranges, "cert_base": cert_base + c0,
            "first": np.ascontiguousarray(cs.cert_first[c0:c1] - f0, dtype=np.uint32),
            "n": np.ascontiguousarray(cs.cert_n[c0:c1], dtype=np.uint32),
            "sigs": cs.sigs[f0:f1], "signer_slots": np.asarray(slots)[cs.signer[f0:f1]], "msgs": cs.msgs[c0:c1]}


def verify_shard(engine, cs, slots, zseed: bytes, rank: int, world: int, cert_base: int = 0):
    """The GPU half of one rank's step: (ranges, cert_ok u8[c1-c0], accepted_stake u64[c1-c0])."""
    sh = shard_inputs(cs, slots, rank, world, cert_base)
    ok, _, st = engine.verify_certs_np(sh["first"], sh["n"], sh["sigs"], sh["signer_slots"], sh["msgs"], zseed,
                                       cert_base=sh["cert_base"])
    return sh["ranges"], ok, st


def verify_sharded(engine, cs, slots, zseed: bytes, rank: int, world: int, group=None, device=None,
                   cert_base: int = 0):
    """Verify this rank's shard of ``cs`` (narwhal_amd.workload.Certificates) on its GPU and
    all-gather the node-wide verdicts.  Returns (cert_ok uint8[C], stake int64[C]) torch tensors on
    ``device`` (default: this rank's GPU)."""
    import torch
    ranges, ok, st = verify_shard(engine, cs, slots, zseed, rank, world, cert_base)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return allgather_verdicts(torch.from_numpy(ok).to(dev), torch.from_numpy(st.astype(np.int64)).to(dev), ranges,
                              group)


def split_bounds(n: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous vote ranges of one batch split over ``world`` ranks."""
    return [((n * r) // world, (n * (r + 1)) // world) for r in range(world)]


def verify_split_batch(engine, msgs, pks, sigs, zseed: bytes, batch_index: int, rank: int, world: int,
                       group=None, device=None) -> bool:
    """One huge batch (e.g. a 6,667-vote certificate at N = 10,000) split across the ranks
    (SURVEY.md §8(e)): each rank evaluates its votes' share of dalek's batch equation
    (nw_verify_batch_partial; coefficients keyed by the vote's index in the whole batch, so no
    transcript exchange is needed), ONE all-gather exchanges the 160-byte partial points and the
    parse/decode flags, and every rank tests the sum for the identity.  The group arithmetic is
    exact, so the verdict equals the unsplit nw_verify_batch verdict."""
    import torch
    import torch.distributed as dist
    row = split_partial_row(engine, msgs, pks, sigs, zseed, batch_index, rank, world)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    buf = torch.from_numpy(row).to(dev)
    gathered = [torch.empty_like(buf) for _ in range(dist.get_world_size(group))]
    dist.all_gather(gathered, buf, group=group)
    return split_verdict(engine, [g.cpu().numpy() for g in gathered])


def split_partial_row(engine, msgs, pks, sigs, zseed: bytes, batch_index: int, rank: int, world: int):
    """This rank's all-gather row for ``verify_split_batch``: uint8[POINT_BYTES + 8] = its partial
    point, then its parse/decode failure flag."""
    from ._lib import POINT_BYTES
    a, b = split_bounds(len(sigs), world)[rank]
    pt, bad = engine.verify_batch_partial(msgs[a:b], pks[a:b], sigs[a:b], zseed, batch_index, a)
    row = np.zeros(POINT_BYTES + 8, np.uint8)
    row[:POINT_BYTES] = np.frombuffer(bytes(pt), np.uint8)
    row[POINT_BYTES] = 1 if bad else 0
    return row


def split_verdict(engine, rows) -> bool:
    """The batch verdict from every rank's row (in rank order): Err if any shard failed to parse or
    decode, else Ok iff the partial points sum to the identity."""
    from ._lib import POINT_BYTES
    if any(int(r[POINT_BYTES]) for r in rows):
        return False
    return engine.points_sum_is_identity([bytes(r[:POINT_BYTES]) for r in rows])
