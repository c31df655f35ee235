"""Benchmark: Ed25519 certificate verification throughput on MI355X (BASELINE.json metric).

Workload (per GPU, weak scaling): BASELINE config C2 — a 100-validator committee and 14,926
certificates x 67 votes = 1,000,042 signatures, inputs resident in HBM.  One "step" = one full
pass of the hot path over that batch: per-vote strict verdicts + per-certificate batch verdicts +
accepted stake (nw_verify_certs_dev), then (N > 1) an RCCL all-gather of the per-shard verdict
bitmaps and stake tallies — the only collective the path has.

Prints ONE JSON line (rank 0).  ``roofline`` is for the dominant kernel (k_verify), timed with
HIP events recorded by libnwcrypto on the launch stream; ``cpu_baseline`` times the oracle's C
restatement of dalek's batch verify (oracle/, "port") on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Ed25519 sigs verified/s (node, 1/2/4/8 GPU); p50 latency per 2f+1 certificate"
# SURVEY.md §8(d) cost model v1 (frozen): FM per signature at n votes per certificate, 100 u32 MADs per FM
COST_MODEL_FM = {3: 1750, 67: 1030, 667: 811, 977: 775, 6667: 644}
MADS_PER_FM = 100


def valu_peak_mad_per_s():
    """Measured v_mad_u64_u32 peak (tools/valu_peak.hip on the box; profiles/r01_valu_peak.json)."""
    path = os.path.join(ROOT, "profiles", "r01_valu_peak.json")
    with open(path) as f:
        for line in f:
            d = json.loads(line)
            if d.get("instr") == "v_mad_u64_u32":
                return d["lane_ops_per_s"]
    raise RuntimeError("no v_mad_u64_u32 entry in " + path)


def traffic_per_launch():
    """HBM bytes per k_verify launch from the committed rocprofv3 PMC pass (or None)."""
    path = os.path.join(ROOT, "profiles", "traffic_k_verify.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def cpu_baseline(cs, com, seconds):
    """Oracle restatement timed on host cores (rank 0, N = 1 only): bounded sample of certificates."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import nw_ref   # C port of dalek's u64 backend (oracle/nw_ref.c)
        kind, impl = "port", "oracle/nw_ref.c (C restatement of ed25519-dalek 1.0.1 u64 backend)"
    except ImportError:
        nw_ref = None
        kind, impl = "port", "oracle/ed25519_oracle.py (pure Python)"
    threads = int(os.environ.get("NW_CPU_THREADS", "16"))
    zseed = bytes(32)
    done_sigs = 0
    done_certs = 0
    t0 = time.perf_counter()
    if nw_ref is not None:
        # batches of certificates handed to the multi-threaded C verifier until the budget is spent
        per_call = 64
        c = 0
        while time.perf_counter() - t0 < seconds:
            sel = [(c + k) % cs.ncerts for k in range(per_call)]
            ok = nw_ref.verify_certs(cs, com, sel, zseed, threads)
            assert all(ok), "CPU baseline rejected an honest certificate"
            done_certs += len(sel)
            done_sigs += int(sum(int(cs.cert_n[x]) for x in sel))
            c += per_call
        cores = threads
    else:
        import ed25519_oracle as o
        while time.perf_counter() - t0 < seconds:
            c = done_certs % cs.ncerts
            f, n = int(cs.cert_first[c]), int(cs.cert_n[c])
            votes = [(bytes(com.pks[cs.signer[f + v]]), bytes(cs.sigs[f + v])) for v in range(n)]
            assert o.crypto_verify_batch(bytes(cs.msgs[c]), votes, zseed, c)
            done_certs += 1
            done_sigs += n
        cores = 1
    dt = time.perf_counter() - t0
    return {"value": done_sigs / dt, "unit": "sigs/s", "cores": cores, "kind": kind,
            "sample": "%d certificates x %d votes of the C2 workload (%d sigs) in %.1f s; %s" % (
                done_certs, int(cs.cert_n[0]), done_sigs, dt, impl)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--validators", type=int, default=100)
    ap.add_argument("--certs", type=int, default=14926)
    ap.add_argument("--votes", type=int, default=67)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-samples", type=int, default=200)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from narwhal_amd import _lib, workload
    eng = _lib.Engine(device=local)
    com = workload.make_committee(args.validators, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    first_cert = rank * args.certs                      # each rank: its own shard of certificates
    cs = workload.make_certificates(com, args.certs, args.votes, eng, first_cert=first_cert)

    dev = torch.device("cuda", local)
    d_sig = torch.from_numpy(cs.sigs).to(dev)
    d_signer = torch.from_numpy(slots[cs.signer].astype(np.int32)).to(dev)
    d_first = torch.from_numpy(cs.cert_first.astype(np.int32)).to(dev)
    d_n = torch.from_numpy(cs.cert_n.astype(np.int32)).to(dev)
    d_msg = torch.from_numpy(cs.msgs).to(dev)
    d_ok = torch.zeros(cs.ncerts, dtype=torch.uint8, device=dev)
    d_flags = torch.zeros(cs.nsigs, dtype=torch.int32, device=dev)
    d_stake = torch.zeros(cs.ncerts, dtype=torch.int64, device=dev)
    from narwhal_amd import shard
    ranges = [(r * args.certs, (r + 1) * args.certs) for r in range(world)]   # node-wide certificate ranges
    zseed = os.urandom(32)

    def step():
        stream = torch.cuda.current_stream().cuda_stream
        eng.verify_certs_dev(cs.ncerts, d_first.data_ptr(), d_n.data_ptr(), cs.nsigs, d_sig.data_ptr(),
                             d_signer.data_ptr(), d_msg.data_ptr(), zseed, first_cert, d_ok.data_ptr(),
                             d_flags.data_ptr(), d_stake.data_ptr(), stream)
        if world > 1:
            shard.allgather_verdicts(d_ok, d_stake, ranges)   # RCCL all_gather of bitmaps + stake

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ok_all = bool(d_ok.all().item())
    if world > 1:
        dist.barrier()
    eng.profile_read()             # discard warmup events
    eng.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.profile_enable(False)
    kms, kn = eng.profile_read()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([1 if ok_all else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok_all = bool(okt.item())
    assert ok_all, "honest workload rejected"

    total_sigs = world * cs.nsigs * args.steps
    value = total_sigs / elapsed

    out = None
    if rank == 0:
        # roofline of k_verify (cost model v1 algorithmic MADs / measured launch time)
        avg_launch_s = (kms / kn) / 1e3 if kn else float("nan")
        fm = COST_MODEL_FM.get(args.votes)
        achieved = (cs.nsigs * fm * MADS_PER_FM / avg_launch_s) / 1e12 if fm else None
        peak = valu_peak_mad_per_s() / 1e12
        traffic = traffic_per_launch()
        roofline = {"bound": "valu", "kernel": "k_verify", "achieved": achieved, "peak": peak, "unit": "TMAD/s",
                    "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                    "avg_launch_ms": avg_launch_s * 1e3, "launches": kn,
                    "note": "achieved = sigs/launch x %s FM/sig (SURVEY §8(d) cost model v1, n=%d) x 100 u32 "
                            "MADs / avg k_verify time; peak = measured v_mad_u64_u32 rate" % (fm, args.votes)}
        # single-certificate latency (H2D -> kernels -> D2H), the Core::run usage pattern
        lat = []
        for i in range(args.latency_samples):
            c = i % cs.ncerts
            f, n = int(cs.cert_first[c]), int(cs.cert_n[c])
            t1 = time.perf_counter()
            cok, _, _ = eng.verify_certs_np(np.array([0], np.uint32), np.array([n], np.uint32), cs.sigs[f:f + n],
                                            slots[cs.signer[f:f + n]], cs.msgs[c:c + 1], zseed, first_cert + c)
            lat.append(time.perf_counter() - t1)
            assert cok[0] == 1
        lat.sort()
        out = {
            "metric": METRIC, "value": value, "unit": "sigs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (GPU-signed RFC 8032 signatures over SHA-512 certificate digests)",
            "config": {"workload": "C2: %d-validator committee, %d certificates x %d votes (%d sigs) per GPU"
                                   % (args.validators, args.certs, args.votes, cs.nsigs),
                       "validators": args.validators, "certs_per_gpu": args.certs, "votes_per_cert": args.votes,
                       "parallelism": "certificate shards per GPU; RCCL all_gather of verdict bitmaps + stake"},
            "p50_cert_latency_ms": lat[len(lat) // 2] * 1e3, "p99_cert_latency_ms": lat[int(len(lat) * 0.99)] * 1e3,
            "roofline": roofline,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cs, com, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
