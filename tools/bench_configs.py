"""Per-config measurements on ONE MI355X for every BASELINE.json config.

bench.py measures the headline line (C2).  This tool measures the other configs at one GPU's share
of the node load, with the C restatement of dalek (oracle/nw_ref.c) timed beside it and the GPU
verdicts checked against it:

  C1  4 validators, 10,000 certificates x 3 votes (the reference's CPU case; GPU shown for scale)
  C3  1,000 validators, one round = 1,000 certificates x 667 votes (node round on one GPU)
  C4  10,000 validators, 1,250 certificates x 6,667 votes (one GPU's eighth of a node round)
  C5  C3 with 1% adversarial signatures (classes (ii), (iii), (v), (vi), (vii)/(ix) of §8(c))
  W   the worker's simulated load: 100,000 fixed keys, 8-byte messages, 64 verify_batch chunks
      per batch (worker/src/processor.rs:46-81), one nw_verify_batches call per batch

Each line: {"config", "sigs_per_s", "ms_per_step", "p50_cert_latency_ms", "cpu": {...}, "parity": {...}}.
Usage (GPU box): python tools/bench_configs.py [--only C1,C3,...] > gpurun_out/configs.jsonl
"""
import argparse
import hashlib
import json
import os
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

L = 2**252 + 27742317777372353535851937790883648493
STREAMS = 3   # batches in flight (bench.py --streams; 3 vs 2: C5 545 vs 513 M, C3 685 vs 662 M, r04cc)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def time_gpu(eng, cs, slots, zseed, steps, warmup, cert_base=0, streams=2):
    """ms per step with ``streams`` batches in flight (step i on stream i mod S, its own outputs);
    the verdicts and flags returned are checked identical across the output sets."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    d_sig = torch.from_numpy(cs.sigs).to(dev)
    d_signer = torch.from_numpy(slots[cs.signer].astype(np.int32)).to(dev)
    d_first = torch.from_numpy(cs.cert_first.astype(np.int32)).to(dev)
    d_n = torch.from_numpy(cs.cert_n.astype(np.int32)).to(dev)
    d_msg = torch.from_numpy(cs.msgs).to(dev)
    outs = [(torch.zeros(cs.ncerts, dtype=torch.uint8, device=dev), torch.zeros(cs.nsigs, dtype=torch.int32, device=dev),
             torch.zeros(cs.ncerts, dtype=torch.int64, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
            for _ in range(streams)]
    sts = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(streams - 1)]
    n = [0]

    def step():
        d_ok, d_flags, d_stake, d_status = outs[n[0] % streams]
        st = sts[n[0] % streams]
        n[0] += 1
        eng.verify_certs_dev(cs.ncerts, d_first.data_ptr(), d_n.data_ptr(), cs.nsigs, d_sig.data_ptr(),
                             d_signer.data_ptr(), d_msg.data_ptr(), zseed, cert_base, d_ok.data_ptr(),
                             d_flags.data_ptr(), d_stake.data_ptr(), st.cuda_stream, d_status=d_status.data_ptr())

    for _ in range(max(warmup, streams)):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ok = outs[0][0].cpu().numpy().astype(bool)
    flags = outs[0][1].cpu().numpy()
    for o in outs[1:]:
        assert (o[0].cpu().numpy().astype(bool) == ok).all() and (o[1].cpu().numpy() == flags).all()
    return dt, ok, flags


def latency(eng, cs, slots, zseed, samples=50):
    lat = []
    for i in range(samples):
        c = i % cs.ncerts
        f, n = int(cs.cert_first[c]), int(cs.cert_n[c])
        t1 = time.perf_counter()
        eng.verify_certs_np(np.array([0], np.uint32), np.array([n], np.uint32), cs.sigs[f:f + n],
                            slots[cs.signer[f:f + n]], cs.msgs[c:c + 1], zseed, c)
        lat.append(time.perf_counter() - t1)
    lat.sort()
    return lat[len(lat) // 2] * 1e3


def cpu_rate(cs, com, zseed, seconds, threads):
    import nw_ref
    done = 0
    c = 0
    t0 = time.perf_counter()
    per = max(1, min(cs.ncerts, 4 * threads))
    while time.perf_counter() - t0 < seconds:
        sel = [(c + k) % cs.ncerts for k in range(per)]
        nw_ref.verify_certs(cs, com, sel, zseed, threads)
        done += int(sum(int(cs.cert_n[x]) for x in sel))
        c += per
    dt = time.perf_counter() - t0
    return {"sigs_per_s": done / dt, "threads": threads, "sample_sigs": done, "seconds": dt,
            "impl": "oracle/nw_ref.c (C restatement of ed25519-dalek 1.0.1 u64 backend)"}


def parity_certs(cs, com, ok_gpu, zseed, sel, threads):
    import nw_ref
    want = nw_ref.verify_certs(cs, com, sel, zseed, threads)
    got = [bool(ok_gpu[c]) for c in sel]
    return {"certs_checked": len(sel), "mismatches": int(sum(a != b for a, b in zip(got, want))),
            "rejected": int(sum(1 for w in want if not w))}


# ------------------------------------------------------------------------------ adversarial mix
def secret_scalar(seed):
    h = hashlib.sha512(seed).digest()
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def make_adversarial(cs, com, frac, rng):
    """Replace ``frac`` of the signatures with a uniform mix of §8(c) classes (keys stay honest):
    ii   R = identity, S = k a            (strict reject, batch accept)
    iii  R' = R + T8, S = r + k' a         (strict reject; batch accept iff 8 | z)
    v    S + l                             (reject)
    vi   S with the top bits set           (reject)
    vii  R with a flipped bit              (undecodable or mismatching: reject)
    ix   signature of another message      (reject)"""
    import ed25519_oracle as o
    n = cs.nsigs
    idx = rng.choice(n, size=int(n * frac), replace=False)
    sigs = cs.sigs.copy()
    classes = ["ii", "iii", "v", "vi", "vii", "ix"]
    t8 = o.small_order_generator()
    cert_of = np.repeat(np.arange(cs.ncerts), cs.cert_n.astype(np.int64))
    kinds = {}
    for j, i in enumerate(idx):
        cls = classes[j % len(classes)]
        kinds[int(i)] = cls
        seed = bytes(com.seeds[cs.signer[i]])
        pk = bytes(com.pks[cs.signer[i]])
        msg = bytes(cs.msgs[cert_of[i]])
        s = bytearray(sigs[i])
        if cls == "ii":
            R = (1).to_bytes(32, "little")
            a, _ = secret_scalar(seed)
            k = int.from_bytes(hashlib.sha512(R + pk + msg).digest(), "little") % L
            s = bytearray(R + (k * a % L).to_bytes(32, "little"))
        elif cls == "iii":
            a, prefix = secret_scalar(seed)
            r = int.from_bytes(hashlib.sha512(prefix + msg).digest(), "little") % L
            Rp = o.pt_compress(o.pt_add(o.pt_mul(r, o.B_POINT), t8))
            k = int.from_bytes(hashlib.sha512(Rp + pk + msg).digest(), "little") % L
            s = bytearray(Rp + ((r + k * a) % L).to_bytes(32, "little"))
        elif cls == "v":
            sv = int.from_bytes(bytes(s[32:]), "little") + L
            s[32:] = sv.to_bytes(32, "little")
        elif cls == "vi":
            s[63] |= 0xE0
        elif cls == "vii":
            s[rng.integers(0, 31)] ^= 1 << int(rng.integers(0, 8))
        else:
            s = bytearray(o.sign(seed, msg[::-1]))
        sigs[i] = np.frombuffer(bytes(s), np.uint8)
    cs.sigs = sigs
    return kinds


# ------------------------------------------------------------------------------ configs
def run_cert_config(name, eng_factory, validators, ncerts, votes, steps, warmup, cpu_seconds, threads,
                    adversarial=0.0, parity_sample=64, streams=None):
    from narwhal_amd import workload
    eng = eng_factory()
    t0 = time.perf_counter()
    com = workload.make_committee(validators, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    t_keys = time.perf_counter() - t0
    cs = workload.make_certificates(com, ncerts, votes, eng)
    kinds = {}
    if adversarial:
        kinds = make_adversarial(cs, com, adversarial, np.random.default_rng(5))
    zseed = bytes(range(32))
    dt1, _, _ = time_gpu(eng, cs, slots, zseed, steps, warmup, streams=1)
    streams = STREAMS if streams is None else streams
    dt, ok, flags = time_gpu(eng, cs, slots, zseed, steps, warmup, streams=streams)
    sel = list(range(0, ncerts, max(1, ncerts // parity_sample)))[:parity_sample]
    out = {"config": name, "validators": validators, "certs": ncerts, "votes_per_cert": votes,
           "sigs_per_step": int(cs.nsigs), "key_window": eng.key_window(), "committee_load_s": t_keys,
           "ms_per_step": dt * 1e3, "sigs_per_s": cs.nsigs / dt, "batches_in_flight": streams,
           "ms_per_step_serial": dt1 * 1e3, "sigs_per_s_serial": cs.nsigs / dt1,
           "certs_accepted": int(ok.sum()), "p50_cert_latency_ms": latency(eng, cs, slots, zseed)}
    out["parity"] = parity_certs(cs, com, ok, zseed, sel, threads)
    if kinds:
        import nw_ref
        cert_of = np.repeat(np.arange(cs.ncerts), cs.cert_n.astype(np.int64))
        strict_bad = 0
        for i, cls in kinds.items():
            want = nw_ref.verify_strict(bytes(com.pks[cs.signer[i]]), bytes(cs.msgs[cert_of[i]]), bytes(cs.sigs[i]))
            got = bool(flags[i] & 0x8)
            strict_bad += int(want != got)
        out["parity"]["adversarial_sigs"] = len(kinds)
        out["parity"]["strict_mismatches"] = strict_bad
        out["slow_path_sigs"] = int(((flags & 0x1000) != 0).sum())
    if cpu_seconds > 0:
        out["cpu"] = cpu_rate(cs, com, zseed, cpu_seconds, threads)
        out["gpu_over_cpu"] = out["sigs_per_s"] / out["cpu"]["sigs_per_s"]
    del eng
    return out


def run_worker(eng_factory, n_keys, per_batch, steps, cpu_seconds, threads):
    """worker/src/processor.rs:46-81 with enable_verification: keys fixed at spawn; each batch
    re-verifies min(100k, #tx) signatures as 64 verify_batch chunks."""
    from narwhal_amd import workload
    eng = eng_factory()
    seeds = np.frombuffer(workload._chacha20_keystream(32 * n_keys), np.uint8).reshape(n_keys, 32).copy()
    msgs = np.zeros((n_keys, 8), np.uint8)
    msgs[:] = np.arange(n_keys, dtype="<u8").view(np.uint8).reshape(n_keys, 8)
    t0 = time.perf_counter()
    pks, sigs = eng.sign_many_np(seeds, msgs)
    slots = eng.committee_load_np(pks)
    t_keys = time.perf_counter() - t0
    count = per_batch
    chunks = [((count * c) // 64, min(count, (count * (c + 1)) // 64) - (count * c) // 64) for c in range(64)]
    first = np.array([f for f, _ in chunks], np.uint32)
    cnts = np.array([n for _, n in chunks], np.uint32)
    zseed = bytes(32)
    eng.verify_batches_np(first, cnts, msgs[:count], slots[:count], sigs[:count], zseed, 0)   # warm
    t0 = time.perf_counter()
    for b in range(steps):
        bok, sok = eng.verify_batches_np(first, cnts, msgs[:count], slots[:count], sigs[:count], zseed, 64 * b)
        assert bok.all() and sok.all()
    dt = (time.perf_counter() - t0) / steps
    out = {"config": "W: worker verify load", "keys": n_keys, "sigs_per_batch": count, "chunks": 64,
           "key_window": eng.key_window(), "key_load_s": t_keys, "ms_per_batch": dt * 1e3,
           "sigs_per_s": count / dt, "note": "host-buffer path (PCIe + ctypes marshalling included)"}
    if cpu_seconds > 0:
        import nw_ref
        done = 0
        t0 = time.perf_counter()
        c = 0
        while time.perf_counter() - t0 < cpu_seconds:
            f, n = chunks[c % 64]
            nw_ref.verify_batch_msgs([bytes(m) for m in msgs[f:f + n]], [bytes(p) for p in pks[f:f + n]],
                                     [bytes(s) for s in sigs[f:f + n]], zseed, c)
            done += n
            c += 1
        dt = time.perf_counter() - t0
        out["cpu"] = {"sigs_per_s": done / dt, "threads": 1, "sample_sigs": done, "seconds": dt,
                      "impl": "oracle/nw_ref.c verify_batch, one chunk at a time on one core"}
    del eng
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C1,C3,C5,C4,W")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("NW_CPU_THREADS", "16")))
    ap.add_argument("--streams", type=int, default=STREAMS)
    args = ap.parse_args()
    globals()["STREAMS"] = max(1, args.streams)
    import torch
    torch.cuda.set_device(0)
    from narwhal_amd import _lib

    def fac():
        return _lib.Engine(device=0, key_window=-1)

    todo = args.only.split(",")
    for name in todo:
        log("config", name)
        if name == "C1":
            r = run_cert_config("C1", fac, 4, 10000, 3, args.steps, 2, args.cpu_seconds, args.threads)
        elif name == "C3":
            r = run_cert_config("C3", fac, 1000, 1000, 667, args.steps, 2, args.cpu_seconds, args.threads)
        elif name == "C5":
            r = run_cert_config("C5", fac, 1000, 1000, 667, args.steps, 2, args.cpu_seconds, args.threads,
                                adversarial=0.01, parity_sample=1000)
        elif name == "C4":
            r = run_cert_config("C4", fac, 10000, 1250, 6667, max(2, args.steps // 2), 1, args.cpu_seconds,
                                args.threads, parity_sample=16, streams=1)   # see bench.py --streams
        elif name == "W":
            r = run_worker(fac, 100000, 62500, args.steps, args.cpu_seconds, args.threads)
        else:
            raise SystemExit("unknown config " + name)
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
