"""Benchmark: Ed25519 certificate verification throughput on MI355X (BASELINE.json metric).

Workload (per GPU, weak scaling): BASELINE config C2 (``configs[1]``) — a 100-validator committee
and 14,926 certificates x 67 votes = 1,000,042 signatures, inputs resident in HBM.  One "step" =
one full pass of the hot path over that batch: per-vote strict verdicts + per-certificate batch
verdicts + accepted stake (nw_verify_certs_dev), then (N > 1) an RCCL all-gather of the per-shard
verdict bitmaps and stake tallies — the only collective the path has.

Prints ONE JSON line (rank 0):
  * ``roofline`` — the dominant kernel, k_verify, timed with HIP events that libnwcrypto records on
    the launch stream around each k_verify launch (nw_profile_*).  ``achieved`` = the kernel's
    algorithmic u32 multiply-accumulates per launch (work model below) / average launch time;
    ``peak`` = the measured v_mad_u64_u32 rate (tools/valu_peak.hip -> profiles/r01_valu_peak.json).
  * ``cpu_baseline`` — the oracle's C restatement of dalek 1.0.1 (oracle/nw_ref.c, "port") timed on
    the host cores on a bounded sample of the same certificates.
  * ``digest`` — the worker's bulk SHA-512 (worker/src/processor.rs:65) over the C4 batch shape
    (bincode batches of 977 x 512-B transactions), GPU vs hashlib on one host core.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Ed25519 sigs verified/s (node, 1/2/4/8 GPU); p50 latency per 2f+1 certificate"
# SURVEY.md §8(d) cost model v1 (frozen): FM per signature of dalek's algorithm at n votes per
# certificate (Straus / Pippenger MSM + R decompression).  Reported as ``dalek_equiv`` only: the
# kernel runs a different (cheaper) algorithm, so v1 is not its work.
COST_MODEL_V1_FM = {3: 1750, 67: 1030, 667: 811, 977: 775, 6667: 644}
MADS_PER_FM = 100          # 10 x 10 radix-2^25.5 limb products per field multiplication
B_WINDOW = 24              # default basepoint comb window (nw_point.h; the library reports its own)
MADD_FM = 7                # mixed (affine Niels) addition = 7 field multiplications


def comb_pos(w):
    return (256 + w - 1) // w


def kverify_fm_per_sig(key_window, base_window=B_WINDOW):
    """k_verify's field multiplications per signature: one mixed addition per comb digit position
    of s (basepoint comb) and of h (key comb); no doublings (nw_core.h comb_sB_minus_hA).  The
    SHA-512 block, mod-l reduction and digit recoding are VALU work not counted here."""
    return MADD_FM * (comb_pos(base_window) + comb_pos(key_window))


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
    """HBM bytes per k_verify launch from the committed rocprofv3 PMC passes (or None)."""
    path = os.path.join(ROOT, "profiles", "traffic_k_verify.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def cpu_baseline(cs, com, seconds):
    """Oracle restatement timed on host cores (rank 0, N = 1 only): bounded sample of certificates."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import nw_ref   # C restatement of dalek's u64 backend (oracle/nw_ref.c); test/baseline only
    threads = int(os.environ.get("NW_CPU_THREADS", "16"))
    zseed = bytes(32)
    done_sigs = done_certs = 0
    per_call = 64
    c = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        sel = [(c + k) % cs.ncerts for k in range(per_call)]
        ok = nw_ref.verify_certs(cs, com, sel, zseed, threads)
        assert all(ok), "CPU baseline rejected an honest certificate"
        done_certs += len(sel)
        done_sigs += int(sum(int(cs.cert_n[x]) for x in sel))
        c += per_call
    dt = time.perf_counter() - t0
    return {"value": done_sigs / dt, "unit": "sigs/s", "cores": threads, "kind": "port",
            "sample": "%d certificates x %d votes of the C2 workload (%d sigs) in %.1f s on %d threads; "
                      "oracle/nw_ref.c (C restatement of ed25519-dalek 1.0.1 u64 backend: per-vote A "
                      "decompression + Straus MSM, as crypto/src/lib.rs:206-219)"
                      % (done_certs, int(cs.cert_n[0]), done_sigs, dt, threads)}


def digest_leg(eng, dev, n_batches, reps, cpu_seconds):
    """Worker batch digests: SHA-512 of n_batches bincode batches resident in HBM (one lane per
    batch: each batch is one sequential compression chain), plus the saturated kernel rate on
    many short messages and hashlib on one host core."""
    import hashlib
    import numpy as np
    import torch
    from narwhal_amd import workload
    out = {}
    host = workload.worker_batches_np(n_batches)
    blen = host.shape[1]
    d_data = torch.from_numpy(host.reshape(-1)).to(dev)
    d_off = torch.arange(n_batches, dtype=torch.int64, device=dev) * blen
    d_len = torch.full((n_batches,), blen, dtype=torch.int64, device=dev)
    d_out = torch.empty((n_batches, 64), dtype=torch.uint8, device=dev)

    def run(nb, d_data, d_off, d_len, d_out, reps):
        st = torch.cuda.current_stream()
        eng.sha512_many_dev(d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), nb, d_out.data_ptr(),
                            st.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            eng.sha512_many_dev(d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), nb, d_out.data_ptr(),
                                st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps / 1e3

    t = run(n_batches, d_data, d_off, d_len, d_out, reps)
    padded = n_batches * ((blen + 17 + 127) // 128) * 128
    got = d_out[:4].cpu().numpy()
    for b in range(4):
        assert bytes(got[b]) == hashlib.sha512(host[b].tobytes()).digest(), "GPU batch digest mismatch"
    out["workload"] = "%d worker batches x %d B (977 x 512-B tx, bincode WorkerMessage::Batch)" % (n_batches, blen)
    out["GBps"] = n_batches * blen / t / 1e9
    out["batches_per_s"] = n_batches / t
    out["kernel_ms"] = t * 1e3
    out["roofline_hbm"] = {"achieved": padded / t / 1e9, "peak": 8000.0, "unit": "GB/s",
                           "frac": padded / t / 1e9 / 8000.0}
    del d_data, d_off, d_len, d_out
    # saturated rate: 2^21 independent 1 KiB messages (enough concurrent chains to fill every SIMD)
    ns, ml = 1 << 21, 1024
    g = torch.Generator(device="cpu").manual_seed(7)
    small = torch.randint(0, 256, (ns * ml,), dtype=torch.uint8, generator=g)
    d_small = small.to(dev)
    s_off = torch.arange(ns, dtype=torch.int64, device=dev) * ml
    s_len = torch.full((ns,), ml, dtype=torch.int64, device=dev)
    s_out = torch.empty((ns, 64), dtype=torch.uint8, device=dev)
    ts = run(ns, d_small, s_off, s_len, s_out, reps)
    chk = s_out[:2].cpu().numpy()
    sm = small[:2 * ml].numpy()
    for b in range(2):
        assert bytes(chk[b]) == hashlib.sha512(sm[b * ml:(b + 1) * ml].tobytes()).digest()
    out["valu_ceiling_GBps"] = ns * ((ml + 17 + 127) // 128) * 128 / ts / 1e9
    out["roofline_valu"] = {"achieved": out["roofline_hbm"]["achieved"], "peak": out["valu_ceiling_GBps"],
                            "unit": "GB/s", "frac": out["roofline_hbm"]["achieved"] / out["valu_ceiling_GBps"],
                            "note": "peak = same kernel on 2^21 x 1 KiB messages (saturated SHA-512 VALU rate)"}
    del d_small, s_off, s_len, s_out
    if cpu_seconds > 0:
        t0 = time.perf_counter()
        nb = 0
        while time.perf_counter() - t0 < cpu_seconds:
            hashlib.sha512(host[nb % n_batches].tobytes()).digest()
            nb += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"GBps": nb * blen / dt / 1e9, "cores": 1, "kind": "hashlib (OpenSSL) SHA-512",
                               "sample": "%d batches in %.1f s" % (nb, dt)}
    return out


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
    ap.add_argument("--digest-batches", type=int, default=10000, help="0 disables the digest leg")
    ap.add_argument("--key-window", type=int, default=-1,
                    help="key comb window; -1 = committee mode (library sizes it for the loaded committee)")
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

    from narwhal_amd import _lib, shard, workload
    eng = _lib.Engine(device=local, key_window=args.key_window)
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
    ok_all = bool(d_ok.all().item()) and bool((d_stake == args.votes).all().item())
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
    kms, kn, ksigs = eng.profile_read()
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

    if rank == 0:
        avg_launch_s = (kms / kn) / 1e3 if kn else float("nan")
        if ksigs is None:                              # library without nw_profile_read_sigs (A/B runs)
            ksigs = cs.nsigs * kn
        sigs_per_launch = ksigs / kn if kn else 0.0
        kw = eng.key_window()
        bw = eng.base_window()
        fm = kverify_fm_per_sig(kw, bw)
        peak = valu_peak_mad_per_s() / 1e12
        achieved = sigs_per_launch * fm * MADS_PER_FM / avg_launch_s / 1e12
        v1 = COST_MODEL_V1_FM.get(args.votes)
        roofline = {
            "bound": "valu", "kernel": "k_verify", "achieved": achieved, "peak": peak, "unit": "TMAD/s",
            "frac": achieved / peak, "traffic": traffic_per_launch(),
            "avg_launch_ms": avg_launch_s * 1e3, "launches": kn,
            "work_model": "%.0f sigs/launch (%d launches per step) x %d FM/sig (7 FM per mixed addition x (%d basepoint "
                          "+ %d key) comb positions, key window %d) x 100 u32 MADs; SHA-512/mod-l/recoding VALU work "
                          "not counted; peak = measured v_mad_u64_u32 rate"
                          % (sigs_per_launch, kn // args.steps, fm, comb_pos(bw), comb_pos(kw), kw),
            "dalek_equiv": {"fm_per_sig": v1, "TMADps": (sigs_per_launch * v1 * MADS_PER_FM / avg_launch_s / 1e12)
                            if v1 else None,
                            "note": "SURVEY §8(d) cost model v1 = dalek's MSM work per signature; the comb "
                                    "algorithm needs %.1fx fewer FM" % (v1 / fm) if v1 else ""},
        }
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
                       "key_window": kw,
                       "parallelism": "certificate shards per GPU; RCCL all_gather of verdict bitmaps + stake"},
            "p50_cert_latency_ms": lat[len(lat) // 2] * 1e3 if lat else None,
            "p99_cert_latency_ms": lat[int(len(lat) * 0.99)] * 1e3 if lat else None,
            "roofline": roofline,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cs, com, args.cpu_seconds)
        else:
            out["cpu_baseline"] = None
        if world == 1 and args.digest_batches > 0:
            del d_sig, d_signer, d_flags
            out["digest"] = digest_leg(eng, dev, args.digest_batches, 3,
                                       0.0 if args.no_cpu_baseline else 3.0)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
