"""Benchmark: Ed25519 certificate verification throughput on MI355X (BASELINE.json metric).

Workload (per GPU, weak scaling): BASELINE config C2 (``configs[1]``) — a 100-validator committee
and 14,926 certificates x 67 votes = 1,000,042 signatures, inputs resident in HBM.  One "step" =
one full pass of the hot path over that batch: per-vote strict verdicts + per-certificate batch
verdicts + accepted stake (nw_verify_certs_dev), then (N > 1) an RCCL all-gather of the per-shard
verdict bitmaps and stake tallies — the only collective the path has.

``python bench.py --gpus N`` with N > 1 and no torch.distributed environment re-launches itself as
N ranks (``torch.distributed.run``, one process per GPU, 127.0.0.1 rendezvous) from a parent that
never touches the GPU; under the driver's own ``torch.distributed.run`` it runs as one rank.

Prints ONE JSON line (rank 0):
  * ``roofline`` — the dominant kernel, k_verify, timed with HIP events that libnwcrypto records on
    the launch stream around each k_verify launch (nw_profile_*).  ``achieved`` = the kernel's
    algorithmic u32 multiply-accumulates per launch (work model below) / average launch time;
    ``peak`` = the measured v_mad_u64_u32 rate (tools/valu_peak.hip -> profiles/r01_valu_peak.json).
  * ``cpu_baseline`` — the oracle's C restatement of dalek 1.0.1 (oracle/nw_ref.c, "port") timed on
    every host core this process may run on, on a bounded sample of the same certificates; the
    per-GPU share of that host (cores / 8 GPUs) is reported beside it.
  * ``host_fed`` — the same C2 certificates through nw_verify_certs from host buffers (PCIe
    included), several calls in flight so copies overlap compute: what the Rust drop-in sees.
  * ``digest`` — the worker's bulk SHA-512 (worker/src/processor.rs:65) over bincode batches of
    977 x 512-B transactions: node load and the C4 per-GPU share, host->device copy included,
    concurrently with a verify step on a second stream, the single-chain bound, and hashlib on
    every host core.
  * ``msm`` — the variable-base Pippenger path (keys outside the committee cache) at the worker's
    load shape: 64 verify_batch chunks of ~977 signatures over fresh keys.
"""
import argparse
import json
import math
import os
import socket
import subprocess
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
GPUS_PER_NODE = 8


def comb_pos(w):
    return (256 + w - 1) // w


def kverify_fm_per_sig(key_window, base_window=B_WINDOW):
    """k_verify's field multiplications per signature, as the kernel executes them: one mixed
    addition per comb digit position of s (basepoint comb) and of h (key comb), no doublings,
    except the chain's first entry, which is converted to extended coordinates with ONE
    multiplication (T = X*Y) instead of being added to the identity (nw_core.h comb_pass_dig<...,
    true, ...>), and the chain's last addition, which skips T = e*h (6 FM, comb_pass_dig<..., LAST>).
    C2 (W24 + W20): 7 x (11 + 13 - 1) + 1 - 1 = 161.  The SHA-512 block, mod-l reduction and digit
    recoding are VALU work not counted here."""
    return MADD_FM * (comb_pos(base_window) + comb_pos(key_window) - 1) + 1 - 1


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


def clock_frac_profile():
    """k_verify's fraction of the MAD peak per shader cycle (both kernels timed in cycles by PMC
    GRBM_GUI_ACTIVE: gpu_pmc.sh passes -> profiles/r05/clock_frac_r05.json; the MAD peak per cycle from
    tools/valu_peak under the same counter, profiles/r04/clock_frac_r04h.json)."""
    path = os.path.join(ROOT, "profiles", "r05", "clock_frac_r05.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return {"frac_per_cycle": d["frac_per_cycle"], "peak_mad_per_cycle": d["peak_mad_per_cycle"],
            "kverify_alg_mad_per_cycle": d["kverify_alg_mad_per_cycle"],
            "source": "profiles/r05/clock_frac_r05.json (PMC GRBM_GUI_ACTIVE on k_verify at C2, same 161-FM work "
                      "model; peak per cycle: tools/valu_peak, profiles/r04/clock_frac_r04h.json)"}


def host_cores():
    """Host threads this process may run on (the whole host unless the scheduler restricts it)."""
    return len(os.sched_getaffinity(0))


def cgroup_cpu_quota():
    """CPUs the container's cgroup may use (cpu.max quota / period), or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def host_topology():
    """(physical cores, logical CPUs) of the whole host, from sysfs topology (a container sees the
    host's CPUs there even when its cgroup quota is far smaller)."""
    import glob
    cores, logical = set(), 0
    for d in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/topology"):
        try:
            with open(os.path.join(d, "physical_package_id")) as f:
                pkg = f.read().strip()
            with open(os.path.join(d, "core_id")) as f:
                core = f.read().strip()
        except OSError:
            continue
        cores.add((pkg, core))
        logical += 1
    if not cores:
        n = os.cpu_count() or 1
        return n, n
    return len(cores), logical


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_thread_candidates():
    """Thread counts worth timing: the cgroup quota and twice it (a quota of q CPUs still lets 2q
    threads overlap their stalls; beyond that they only time-slice), capped by the affinity mask.
    Without a quota: the affinity count."""
    aff = host_cores()
    q = cgroup_cpu_quota()
    if not q:
        return [aff]
    base = max(1, int(math.ceil(q)))
    return sorted({min(aff, base), min(aff, 2 * base)})


def cpu_baseline(cs, com, seconds, probe_seconds=2.5, label="C2", threads=None):
    """Oracle restatement timed on the host cores (rank 0, at every world size, after the timed
    region): bounded sample of certificates.  A short sweep over the candidate thread counts (cpu_thread_candidates; forced
    with NW_CPU_THREADS) picks the host's best rate, which is then timed on the main sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import nw_ref   # C restatement of dalek's u64 backend (oracle/nw_ref.c); test/baseline only
    zseed = bytes(32)
    forced = threads or int(os.environ.get("NW_CPU_THREADS", "0"))
    cands = [forced] if forced else cpu_thread_candidates()

    def run(threads, secs):
        done_sigs = done_certs = 0
        per_call = max(64, 4 * threads)
        c = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            sel = [(c + k) % cs.ncerts for k in range(per_call)]
            ok = nw_ref.verify_certs(cs, com, sel, zseed, threads)
            assert all(ok), "CPU baseline rejected an honest certificate"
            done_certs += len(sel)
            done_sigs += int(sum(int(cs.cert_n[x]) for x in sel))
            c += per_call
        dt = time.perf_counter() - t0
        return done_sigs / dt, done_sigs, done_certs, dt

    sweep = {}
    if len(cands) > 1:
        for t in cands:
            sweep[str(t)] = run(t, probe_seconds)[0]
        threads = max(cands, key=lambda t: sweep[str(t)])
    else:
        threads = cands[0]
    rate, done_sigs, done_certs, dt = run(threads, seconds)
    # The measured slice is the container's CPU quota, not the host.  Per quota CPU (one CPU-second
    # per second of wall time) the rate extrapolates to the host's physical cores (conservative: an
    # SMT sibling is counted as no extra capacity) and, as an upper bound, to its logical CPUs.
    quota = cgroup_cpu_quota()
    slice_cpus = quota if quota else float(threads)
    per_cpu = rate / slice_cpus
    phys, logical = host_topology()
    host_rate = per_cpu * phys
    return {"value": rate, "unit": "sigs/s", "cores": threads, "kind": "port",
            "measured_slice": {"cpus": slice_cpus, "threads": threads,
                               "note": "cgroup CPU quota of this process (the value above is measured on it)"},
            "per_cpu": {"value": per_cpu, "unit": "sigs/s per quota CPU"},
            "host_extrapolated": {"value": host_rate, "physical_cores": phys, "logical_cpus": logical,
                                  "upper_bound_logical": per_cpu * logical,
                                  "note": "EXTRAPOLATED, not measured: per_cpu x the host's physical cores "
                                          "(SMT siblings counted as no extra capacity); upper_bound_logical = "
                                          "per_cpu x logical CPUs"},
            "per_gpu_share": {"value": host_rate / GPUS_PER_NODE, "cores": phys / GPUS_PER_NODE,
                              "note": "host_extrapolated / %d GPUs per node" % GPUS_PER_NODE},
            "cpu_model": cpu_model(),
            # the affinity mask can be far wider than the cgroup's CPU quota (GPU box: 256 vs 16);
            # threads beyond ~2x the quota only time-slice (profiles/r02/cpu_probe_r02.json)
            "cgroup_cpu_quota": cgroup_cpu_quota(), "affinity_cpus": host_cores(),
            "thread_sweep_sigs_per_s": sweep or None,
            "sample": "%d certificates x %d votes of the %s workload (%d sigs) in %.1f s on %d threads (%s); "
                      "oracle/nw_ref.c (C restatement of ed25519-dalek 1.0.1 u64 backend: per-vote A "
                      "decompression + Straus MSM below 190 votes, Pippenger above, as dalek's verify_batch via "
                      "crypto/src/lib.rs:206-219)"
                      % (done_certs, int(cs.cert_n[0]), label, done_sigs, dt, threads,
                         "best of the sweep" if len(cands) > 1 else "thread count given")}


def hashlib_rate(batches, threads, seconds):
    """Host SHA-512 (hashlib / OpenSSL, releases the GIL) over worker batches on ``threads`` threads:
    (bytes/s, batches hashed, seconds)."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    n = batches.shape[0]
    stop = time.perf_counter() + seconds

    def loop(k):
        nb = 0
        while time.perf_counter() < stop:
            hashlib.sha512(batches[(k + nb) % n].data).digest()
            nb += 1
        return nb

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        nb = sum(ex.map(loop, range(threads)))
    dt = time.perf_counter() - t0
    return nb * batches.shape[1] / dt, nb, dt


def cpu_step_with_digests(cb, batches, plan, seconds):
    """C4 on the host: the rank's signatures at the measured verify rate plus its worker-batch
    digests at the measured hashlib rate, both on the same threads (one after the other, as one
    host would have to do both): the CPU counterpart of a C4 step."""
    bps, nb, dt = hashlib_rate(batches, cb["cores"], seconds)
    verify_s = plan["sigs"] / cb["value"]
    digest_s = plan["digest_batches"] * batches.shape[1] / bps
    return {"hash_GBps": bps / 1e9, "hash_sample": "%d batches of %d B in %.1f s on %d threads (hashlib)"
                                                    % (nb, batches.shape[1], dt, cb["cores"]),
            "step_s": verify_s + digest_s, "verify_s": verify_s, "digest_s": digest_s,
            "sigs_per_s": plan["sigs"] / (verify_s + digest_s),
            "note": "per-GPU C4 share (%d sigs + %d batches) done by this host: verify at cpu_baseline.value, then "
                    "the digests at hash_GBps" % (plan["sigs"], plan["digest_batches"])}


def host_fed(eng, cs, slots, zseed, chunks=16, threads=8, reps=5, stream_passes=20):
    """C2 through nw_verify_certs from pageable host buffers (PCIe and host staging included): what a
    Rust caller that hands over host buffers sees.  ``chunks`` calls on ``threads`` host threads (every
    call leases its own workspace and stream, so one call's upload overlaps another's kernels).

    value: STREAMING, the calls of ``stream_passes`` passes submitted back to back on the same threads
    (a node's Core keeps submitting as batches arrive; no barrier between passes), every pass on its
    OWN host arrays, allocated after the warm-up round and touched by no earlier call.  first_round:
    the same streaming round as the very first host-buffer work of the process (the warm-up, on
    separate arrays): copy stalls (calling threads inside hipMemcpyAsync for 5-13 ms while the GPU
    idles: HIP API trace, profiles/r05/host_fed_r05.txt) concentrate there.  passes: the same calls
    with a barrier after every pass (ms_reps), on reused and on freshly allocated buffers."""
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    bounds = np.linspace(0, cs.ncerts, chunks + 1).astype(int)
    parts = []
    for a, b in zip(bounds, bounds[1:]):
        f0, f1 = int(cs.cert_first[a]), int(cs.cert_first[b - 1] + cs.cert_n[b - 1])
        parts.append((cs.cert_first[a:b] - f0, cs.cert_n[a:b], np.ascontiguousarray(cs.sigs[f0:f1]),
                      np.ascontiguousarray(slots[cs.signer[f0:f1]]), np.ascontiguousarray(cs.msgs[a:b]), int(a)))

    def run(p):
        ok, _, _ = eng.verify_certs_np(p[0], p[1], p[2], p[3], p[4], zseed, p[5])
        return bool(ok.all())

    def fresh(ps):   # new host buffers, as a node's network receives would hand over
        return [(a, b, c.copy(), d.copy(), e.copy(), f) for a, b, c, d, e, f in ps]

    warm_sets = [fresh(parts) for _ in range(4)]
    with ThreadPoolExecutor(threads) as ex:
        # the first streaming round of the process (warm-up, timed for the record, its own arrays)
        t0 = time.perf_counter()
        assert all(ex.map(run, [p for k in range(stream_passes) for p in warm_sets[k % len(warm_sets)]]))
        t_first = time.perf_counter() - t0
        del warm_sets
        stream_sets = [fresh(parts) for _ in range(stream_passes)]    # untouched by any call so far
        fresh_sets = [fresh(parts) for _ in range(reps)]
        t0 = time.perf_counter()
        ok = all(ex.map(run, [p for k in range(stream_passes) for p in stream_sets[k]]))
        t_stream = time.perf_counter() - t0
        assert ok
        del stream_sets
        ts, tf = [], []
        for r in range(reps):
            t0 = time.perf_counter()
            ok = all(ex.map(run, parts))
            ts.append(time.perf_counter() - t0)
            assert ok
            t0 = time.perf_counter()
            ok = all(ex.map(run, fresh_sets[r]))
            tf.append(time.perf_counter() - t0)
            assert ok
    ts.sort()
    tf.sort()
    dt = ts[len(ts) // 2]
    return {"value": stream_passes * cs.nsigs / t_stream, "unit": "sigs/s",
            "ms_per_pass_streaming": t_stream / stream_passes * 1e3,
            "first_round": {"value": stream_passes * cs.nsigs / t_first, "ms_per_pass": t_first / stream_passes * 1e3,
                            "note": "the same streaming round as the process's first host-buffer work (the warm-up, "
                                    "4 rotating array sets of its own)"},
            "passes": {"value": cs.nsigs / dt, "ms": dt * 1e3, "ms_reps": [t * 1e3 for t in ts],
                       "fresh_buffers": {"value": cs.nsigs / tf[len(tf) // 2], "ms": tf[len(tf) // 2] * 1e3,
                                         "ms_reps": [t * 1e3 for t in tf]}},
            "note": "nw_verify_certs on pageable host buffers (every input staged through the call's pinned buffer), "
                    "%d calls of ~%d signatures on %d threads; value: %d passes' calls streamed back to back, each "
                    "pass on its own host arrays allocated after the warm-up round and never passed to the library "
                    "before; passes: a barrier after every pass, median of %d (reused arrays; fresh_buffers: newly "
                    "allocated ones); PCIe and host packing included"
                    % (chunks, cs.nsigs // chunks, threads, stream_passes, reps)}


class BatchUploader:
    """C4 with host-resident worker batches (``--batches host``, the default): each step's batches come from
    PAGEABLE host memory, as the worker's Processor receives them (worker/src/processor.rs:63-65).
    ``stage_next`` copies them into one of two pinned buffers with ``threads`` host threads, chunk by
    chunk, and enqueues each chunk's DMA into one of two HBM buffers on a copy stream as soon as the
    chunk is staged; the digests of step i read the buffer step i-1 uploaded (double buffering, as the
    worker's DigestBatcher keeps DEPTH = 2 windows in flight).  Host staging, PCIe and the digests
    are all inside the timed loop."""

    def __init__(self, host_b, dev, threads=8, chunk=32 << 20, nbuf=2, copy_streams=None):
        import torch
        from concurrent.futures import ThreadPoolExecutor
        self.host = host_b.reshape(-1)
        self.n = self.host.shape[0]
        self.chunk = chunk
        self.nbuf = nbuf
        self.pinned = [torch.empty(self.n, dtype=torch.uint8).pin_memory() for _ in range(nbuf)]
        self.pinned_np = [p.numpy() for p in self.pinned]
        self.dev_buf = [torch.empty(self.n, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        # copy_streams[j]: the stream buffer j's DMAs go on.  Given the digest streams (one per buffer),
        # each upload is queued behind the digests that last read its buffer and ahead of the digests
        # that will read it, so stream order alone orders them and no other stream (which HIP may map
        # onto the same in-order hardware queue) is involved
        self.copy_streams = copy_streams or [torch.cuda.Stream(device=dev)] * nbuf
        self.ev_up = [torch.cuda.Event() for _ in range(nbuf)]
        self.ev_read = [None] * nbuf       # last digest launch that read dev_buf[j]
        self.pool = ThreadPoolExecutor(threads)
        self.threads = threads
        self.next = 0                      # buffer the next stage_next fills
        self.stage_s = []
        self.trace = []                    # (buffer, start, wait for the previous DMA, stage + enqueue)

    def _copy(self, j, a, b):
        import numpy as np
        np.copyto(self.pinned_np[j][a:b], self.host[a:b])

    def stage_next(self, read_stream):
        """Stage + upload the next step's batches into buffer self.next.  ``read_stream``: the stream
        on which this step's digests (reading the other buffer) were just launched, or None."""
        import torch
        if read_stream is not None:       # a FRESH event per record: the reader of each buffer
            ev = torch.cuda.Event()
            ev.record(read_stream)
            self.ev_read[self.pending] = ev
        j = self.next
        t0 = time.perf_counter()
        self.ev_up[j].synchronize()        # the previous DMA out of pinned[j] is done
        t1 = time.perf_counter()
        cs = self.copy_streams[j]
        if self.ev_read[j] is not None:
            cs.wait_event(self.ev_read[j])   # the digests that read dev_buf[j] are done
        bounds = list(range(0, self.n, self.chunk)) + [self.n]
        futs = [self.pool.submit(self._copy, j, a, b) for a, b in zip(bounds, bounds[1:])]
        with torch.cuda.stream(cs):
            for f, a, b in zip(futs, bounds, bounds[1:]):
                f.result()
                self.dev_buf[j][a:b].copy_(self.pinned[j][a:b], non_blocking=True)
        self.ev_up[j].record(cs)
        t2 = time.perf_counter()
        self.stage_s.append(t2 - t0)
        self.trace.append((j, t0, t1 - t0, t2 - t1))
        self.pending = j
        self.next = (j + 1) % self.nbuf

    def ready_buffer(self, stream):
        """The buffer the last stage_next uploaded, ordered after its upload on ``stream``."""
        stream.wait_event(self.ev_up[self.pending])
        return self.dev_buf[self.pending]

    def stats(self):
        st = sorted(self.stage_s[1:]) or [0.0]
        t0 = self.trace[0][1] if self.trace else 0.0
        return {"host_threads": self.threads, "chunk_MiB": self.chunk >> 20,
                "stage_and_enqueue_ms_p50": st[len(st) // 2] * 1e3,
                "trace_ms": [[j, round((t - t0) * 1e3, 2), round(w * 1e3, 2), round(c * 1e3, 2)]
                             for j, t, w, c in self.trace[-12:]],
                "note": "host time per step to copy %d MB from pageable into pinned memory (the DMAs overlap it "
                        "chunk by chunk)" % (self.n // 10 ** 6)}


def digest_leg(eng, dev, n_node, n_share, reps, cpu_seconds, verify_step):
    """Worker batch digests (worker/src/processor.rs:65), one lane per batch (each batch is one
    sequential SHA-512 compression chain)."""
    import hashlib
    import torch
    from narwhal_amd import workload
    out = {}
    host = workload.worker_batches_np(n_node)
    blen = host.shape[1]
    blocks = (blen + 17 + 127) // 128
    st = torch.cuda.current_stream()

    def dev_bufs(nb):
        d_off = torch.arange(nb, dtype=torch.int64, device=dev) * blen
        d_len = torch.full((nb,), blen, dtype=torch.int64, device=dev)
        d_out = torch.empty((nb, 64), dtype=torch.uint8, device=dev)
        return d_off, d_len, d_out

    def timed(fn, reps, stream):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps / 1e3

    def dig(nb, d_data, d_off, d_len, d_out, stream):
        return lambda: eng.sha512_many_dev(d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), nb,
                                           d_out.data_ptr(), stream.cuda_stream)

    d_data = torch.from_numpy(host.reshape(-1)).to(dev)
    d_off, d_len, d_out = dev_bufs(n_node)
    t = timed(dig(n_node, d_data, d_off, d_len, d_out, st), reps, st)
    got = d_out[:4].cpu().numpy()
    for b in range(4):
        assert bytes(got[b]) == hashlib.sha512(host[b].tobytes()).digest(), "GPU batch digest mismatch"
    padded = n_node * blocks * 128
    out["workload"] = "%d worker batches x %d B (977 x 512-B tx, bincode WorkerMessage::Batch)" % (n_node, blen)
    out["kernel"] = ("k_sha512_split2 (one lane pair per batch, two schedule waves)" if n_node <= 32768
                     else "k_sha512_many (one lane per batch)")
    out["GBps"] = n_node * blen / t / 1e9
    out["kernel_ms"] = t * 1e3
    out["roofline_hbm"] = {"achieved": padded / t / 1e9, "peak": 8000.0, "unit": "GB/s",
                           "frac": padded / t / 1e9 / 8000.0}
    # single-chain bound: one batch alone on the GPU (7 separately timed launches: a lone wave's
    # clock varies launch to launch, so the median and the best are both reported)
    lone = sorted(timed(dig(1, d_data, d_off[:1], d_len[:1], d_out, st), 1, st) for _ in range(7))
    t1 = lone[len(lone) // 2]
    out["single_chain"] = {"blocks_per_batch": blocks, "lone_batch_ms": t1 * 1e3, "ns_per_block": t1 / blocks * 1e9,
                           "best_ns_per_block": lone[0] / blocks * 1e9, "lone_batch_ms_all": [x * 1e3 for x in lone],
                           "note": "one batch alone on the GPU, median of 7 launches: a batch is one sequential chain "
                                   "of %d compressions" % blocks}
    # C4 per-GPU share: 1,250 batches; alone, with the host->device copy from pinned memory, and
    # concurrently with the C2 verify step on a second stream
    pinned = torch.from_numpy(host[:n_share].reshape(-1)).pin_memory()
    d_share = torch.empty(pinned.shape, dtype=torch.uint8, device=dev)
    s_off, s_len, s_out = dev_bufs(n_share)
    ts = timed(dig(n_share, d_share, s_off, s_len, s_out, st), reps, st)

    def h2d_and_digest():
        d_share.copy_(pinned, non_blocking=True)
        dig(n_share, d_share, s_off, s_len, s_out, st)()

    th = timed(h2d_and_digest, reps, st)
    assert bytes(s_out[n_share - 1].cpu().numpy()) == hashlib.sha512(host[n_share - 1].tobytes()).digest()
    s2 = torch.cuda.Stream(device=dev)
    tv = timed(lambda: verify_step(st), reps, st)

    def both():
        with torch.cuda.stream(s2):
            d_share.copy_(pinned, non_blocking=True)
            dig(n_share, d_share, s_off, s_len, s_out, s2)()
        verify_step(st)

    torch.cuda.synchronize()
    both()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        both()
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t0) / reps
    out["c4_share"] = {"batches": n_share, "kernel_ms": ts * 1e3, "GBps": n_share * blen / ts / 1e9,
                       "with_h2d_ms": th * 1e3, "with_h2d_GBps": n_share * blen / th / 1e9,
                       "verify_step_ms": tv * 1e3, "overlapped_ms": tb * 1e3,
                       "overlap_saving_ms": (th + tv - tb) * 1e3,
                       "note": "overlapped = H2D + digest of the share on a second stream concurrently with "
                               "one C2 verify step (1,000,042 sigs) on the first"}
    del d_data, d_off, d_len, d_out, d_share, pinned
    # saturated rate: 2^21 independent 1 KiB messages (enough concurrent chains to fill every SIMD)
    ns, ml = 1 << 21, 1024
    g = torch.Generator(device="cpu").manual_seed(7)
    small = torch.randint(0, 256, (ns * ml,), dtype=torch.uint8, generator=g)
    d_small = small.to(dev)
    q_off = torch.arange(ns, dtype=torch.int64, device=dev) * ml
    q_len = torch.full((ns,), ml, dtype=torch.int64, device=dev)
    q_out = torch.empty((ns, 64), dtype=torch.uint8, device=dev)
    tq = timed(dig(ns, d_small, q_off, q_len, q_out, st), reps, st)
    chk = q_out[:2].cpu().numpy()
    sm = small[:2 * ml].numpy()
    for b in range(2):
        assert bytes(chk[b]) == hashlib.sha512(sm[b * ml:(b + 1) * ml].tobytes()).digest()
    out["valu_ceiling_GBps"] = ns * ((ml + 17 + 127) // 128) * 128 / tq / 1e9
    out["roofline_valu"] = {"achieved": out["roofline_hbm"]["achieved"], "peak": out["valu_ceiling_GBps"],
                            "unit": "GB/s", "frac": out["roofline_hbm"]["achieved"] / out["valu_ceiling_GBps"],
                            "note": "peak = k_sha512_many on 2^21 x 1 KiB messages (saturated SHA-512 VALU rate)"}
    del d_small, q_off, q_len, q_out
    if cpu_seconds > 0:
        threads = max(cpu_thread_candidates())
        bps, nb, dt = hashlib_rate(host, threads, cpu_seconds)
        out["cpu_baseline"] = {"GBps": bps / 1e9, "cores": threads, "kind": "hashlib (OpenSSL) SHA-512",
                               "per_gpu_share_GBps": bps / 1e9 / GPUS_PER_NODE,
                               "sample": "%d batches in %.1f s on %d threads" % (nb, dt, threads)}
    return out


def worker_digest_leg(eng, n_batches=1250, windows=(32, 128, 1250), depth=2):
    """The worker's Processor digests (worker/src/processor.rs:63-97) through the batched
    asynchronous path (narwhal_amd.worker.DigestBatcher -> nw_sha512_many_async), host buffers:
    C4's per-GPU share of 508,052-B batches arriving back to back.  Per window size: batches/s and
    the per-batch latency from push to delivery; beside it the one-batch call and one host core
    with hashlib (the reference's serial loop)."""
    import hashlib
    from narwhal_amd import worker, workload
    host = workload.worker_batches_np(n_batches)
    blen = host.shape[1]
    rows = [host[i] for i in range(n_batches)]
    out = {"batches": n_batches, "batch_bytes": blen, "depth": depth, "windows": {}}
    for win in windows:
        b = worker.DigestBatcher(eng, window=win, depth=depth)
        # warm: depth + 2 windows, so every workspace the timed run can lease exists and is sized (a
        # workspace's first use pays its pinned-buffer allocation and first DMAs, ~20 ms)
        for d, x in b.pipeline([rows[k % n_batches] for k in range((depth + 2) * win)]):
            pass
        rows = [r.copy() for r in rows]   # fresh host buffers, as a worker's received batches are
        t_push = {}
        lat = []
        t0 = time.perf_counter()
        for k, x in enumerate(rows):
            t_push[id(x)] = time.perf_counter()
            b.push(x)
            for d, y in b.ready():
                lat.append(time.perf_counter() - t_push[id(y)])
        for d, y in b.drain():
            lat.append(time.perf_counter() - t_push[id(y)])
        dt = time.perf_counter() - t0
        assert len(lat) == n_batches
        lat.sort()
        out["windows"][str(win)] = {"batches_per_s": n_batches / dt, "GBps": n_batches * blen / dt / 1e9,
                                    "p50_latency_ms": lat[len(lat) // 2] * 1e3, "p99_latency_ms": lat[int(len(lat) * 0.99)] * 1e3,
                                    "submissions": b.submissions}
    last = worker.DigestBatcher(eng, window=1, depth=1)
    one = []
    for k in range(7):
        t1 = time.perf_counter()
        last.push(rows[k])
        (d, _), = last.drain()
        one.append(time.perf_counter() - t1)
        assert d == hashlib.sha512(rows[k].tobytes()).digest()
    one.sort()
    t1 = time.perf_counter()
    for k in range(40):
        hashlib.sha512(rows[k].data).digest()
    core = (time.perf_counter() - t1) / 40
    out["one_batch_call_ms"] = {"p50": one[3] * 1e3, "min": one[0] * 1e3}
    out["host_1core"] = {"ms_per_batch": core * 1e3, "batches_per_s": 1.0 / core, "kind": "hashlib (OpenSSL) SHA-512"}
    out["note"] = ("latency = push -> delivery of (digest, batch) in arrival order, all batches available at once; "
                   "a batch's digest is one chain of %d compressions, so no window delivers one sooner than the "
                   "lone-chain time" % ((blen + 17 + 127) // 128))
    return out


def msm_leg(eng, n_sigs=62500, chunks=64, reps=11):
    """Keys outside the committee cache (the worker's direct verify_batch, worker/src/processor.rs:
    75-79, without loading its keys): nw_verify_batches_pk -> Pippenger MSM, host buffers."""
    import numpy as np
    from narwhal_amd import workload
    seeds = np.frombuffer(workload._chacha20_keystream(32 * n_sigs), np.uint8).reshape(n_sigs, 32)
    seeds = seeds[::-1].copy()   # not the committee's keys
    msgs = np.arange(n_sigs, dtype="<u8").view(np.uint8).reshape(n_sigs, 8).copy()
    pks, sigs = eng.sign_many_np(seeds, msgs)
    counts = [min(n_sigs, (n_sigs * (c + 1)) // chunks) - (n_sigs * c) // chunks for c in range(chunks)]
    zseed = os.urandom(32)
    call = eng.prepare_batches_pk_call(counts, msgs, pks, sigs)   # marshalled once, as a Rust caller
    assert call(zseed, 0).all(), "MSM path rejected honest batches"
    times = []
    for r in range(reps):
        t0 = time.perf_counter()
        ok = call(zseed, chunks * (r + 1))
        times.append(time.perf_counter() - t0)
        assert ok.all()
    dt = sorted(times)[len(times) // 2]
    return {"value": n_sigs / dt, "unit": "sigs/s", "ms": dt * 1e3, "ms_all": [t * 1e3 for t in times],
            "workload": "%d verify_batch chunks, %d sigs, 8-byte messages, fresh (uncached) keys" % (chunks, n_sigs),
            "note": "median of %d one-call samples (marshalled once); host buffers incl. PCIe upload and host "
                    "staging; per-kernel times in profiles/r03/" % reps}


def launch_ranks(args, argv):
    """--gpus N outside torch.distributed: one rank per GPU via torch.distributed.run, started from
    this process before it touches the GPU; returns the launcher's exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# BASELINE.json configs a bench run can execute on N ranks (one process per GPU).  "rank" scope:
# the shape is per GPU (weak scaling: C2 = configs[1]; C4 = configs[3], one GPU's eighth of a
# 10,000-validator node round plus the rank's worker-batch digests).  "node" scope: the shape is
# the node's round, partitioned over the ranks by shard.partition (strong scaling: C3 =
# configs[2], 1,000 certificates x 667 votes; config/src/lib.rs:189-194 gives the 2f+1 = 667).
CONFIGS = {
    "C2": {"validators": 100, "certs": 14926, "votes": 67, "scope": "rank", "digest_batches": 0, "streams": 1,
           "baseline": "configs[1]: 100-validator committee, 67-vote certificates, 1M signatures per MI355X"},
    "C3": {"validators": 1000, "certs": 1000, "votes": 667, "scope": "node", "digest_batches": 0, "streams": 3,
           "baseline": "configs[2]: 1,000-validator committee, 667-vote certificates, sharded over the GPUs "
                       "with an RCCL verdict all-gather"},
    "C4": {"validators": 10000, "certs": 1250, "votes": 6667, "scope": "rank", "digest_batches": 1250, "streams": 1,
           "baseline": "configs[3]: 10,000-validator committee, 6,667-vote certificates plus worker 500 KB batch "
                       "SHA-512 digests; per GPU 1/8 of a node round (1,250 certificates, 1,250 batches)"},
}


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS),
                    help="BASELINE config of the timed step (default C2, the headline)")
    ap.add_argument("--validators", type=int, default=None, help="override the config's committee size")
    ap.add_argument("--certs", type=int, default=None, help="override the config's certificate count")
    ap.add_argument("--votes", type=int, default=None, help="override the config's votes per certificate")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-samples", type=int, default=200)
    ap.add_argument("--digest-batches", type=int, default=10000, help="0 disables the digest leg")
    ap.add_argument("--digest-share", type=int, default=1250, help="C4 per-GPU batch share")
    ap.add_argument("--no-extras", action="store_true", help="headline only (no host_fed / msm / latency legs)")
    ap.add_argument("--streams", type=int, default=None,
                    help="batches in flight: step i runs on stream i mod S with its own output buffers, so one "
                         "batch's k_finish / slow path overlaps the next batch's k_verify (1: strictly serial). "
                         "Default per config: 3 for C3 (+14%% over one, r04cc); 1 for C2, where two in flight gain 1.6%% "
                         "(r04p) but the timed k_verify launches then overlap each other and the roofline "
                         "measures shared time (frac 0.40-0.45 instead of ~0.47); 1 for C4, where two 8.3M-signature "
                         "k_verify launches over 10,000 key tables slow each other down (r04o: 401 vs 466 M sigs/s)")
    ap.add_argument("--batches", choices=("host", "hbm"), default="host",
                    help="C4: where the worker batches start each step.  host (default): in pageable host memory, "
                         "as the Processor receives them (worker/src/processor.rs:63-65); host threads stage them "
                         "into pinned buffers and DMA them to HBM inside the timed loop (step i hashes what step "
                         "i-1 uploaded while it stages and uploads step i+1's batches).  hbm: resident in HBM "
                         "(round 4's C4 line, PCIe excluded)")
    ap.add_argument("--digest-join", action="store_true",
                    help="C4: end every step when its digests end (round 4's structure).  Default: the digests "
                         "of consecutive steps overlap (two alternating high-priority digest streams; step i+1's "
                         "digests start when step i's verify kernels end), so a batch's serial SHA-512 chain "
                         "bounds its latency but not the step")
    ap.add_argument("--timing-only", action="store_true", help=argparse.SUPPRESS)   # A/B of timing-only variants
    ap.add_argument("--hw-queues", type=int, default=0, help="set GPU_MAX_HW_QUEUES (1..32) before HIP starts")
    ap.add_argument("--c4-steps", type=int, default=8,
                    help="C2 runs: timed steps of the C4 leg (the north-star config, configs[3]) run after the C2 "
                         "engine is closed; 0 disables it")
    ap.add_argument("--c4-warmup", type=int, default=2)
    ap.add_argument("--cpu-latency-samples", type=int, default=100,
                    help="calls per one-thread CPU latency comparator (cpu_baseline.latency)")
    ap.add_argument("--engine-flags", type=lambda x: int(x, 0), default=0, help=argparse.SUPPRESS)   # nw_opts.flags (A/B)
    ap.add_argument("--key-window", type=int, default=-1,
                    help="key comb window; -1 = committee mode (library sizes it for the loaded committee)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks meet over gloo, rank 0 prints the world")
    a = ap.parse_args(argv)
    if a.hw_queues and not 1 <= a.hw_queues <= 32:
        ap.error("--hw-queues must be in 1..32 (the GPU box refuses GPU_MAX_HW_QUEUES above 32)")
    return a


def config_plan(args, world, rank):
    """The rank's share of the configured step (pure host logic; the dry run prints it)."""
    from narwhal_amd import shard
    c = dict(CONFIGS[args.config])
    validators = args.validators or c["validators"]
    certs = args.certs or c["certs"]
    votes = args.votes or c["votes"]
    if c["scope"] == "node":
        ranges = shard.partition([votes] * certs, world)
        scaling = "strong"
    else:
        ranges = [(r * certs, (r + 1) * certs) for r in range(world)]
        scaling = "weak"
    c0, c1 = ranges[rank]
    return {"config": args.config, "validators": validators, "votes": votes, "node_certs": ranges[-1][1],
            "ranges": ranges, "first_cert": c0, "ncerts": c1 - c0, "sigs": (c1 - c0) * votes,
            "total_sigs": ranges[-1][1] * votes, "digest_batches": c["digest_batches"], "scaling": scaling,
            "baseline": c["baseline"]}


def dry_run(args):
    """Rank plumbing of ``--gpus N`` on CPU (tests/test_bench_launch.py): one gloo all_gather of
    the rank ids and of each rank's workload plan, the same barrier/max-over-ranks pattern as the
    timed loop, one JSON line."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    plan = config_plan(args, world, rank)
    mine = torch.tensor([rank, plan["first_cert"], plan["ncerts"], plan["sigs"], plan["digest_batches"]],
                        dtype=torch.int64)
    got = [torch.zeros(5, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(got, mine)
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    else:
        got = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "gpus_arg": args.gpus, "config": args.config,
                          "ranks": [int(g[0].item()) for g in got],
                          "shards": [{"first_cert": int(g[1]), "ncerts": int(g[2]), "sigs": int(g[3]),
                                      "digest_batches": int(g[4])} for g in got],
                          "total_sigs": plan["total_sigs"], "scaling": plan["scaling"],
                          "local_ranks_env": os.environ.get("LOCAL_RANK")}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def timeit_once(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def latency_legs(eng, com, slots, cs, samples, keep=None):
    """One-call latencies of the paths the Rust shim calls, host buffers, the
    call marshalled once so only the ABI call is timed:
      * strict: crypto::Signature::verify (crypto/src/lib.rs:200-204) -> nw_verify_strict, one
        header/vote signature (primary/src/core.rs:313,335), key in the committee cache and not;
      * batch: crypto::Signature::verify_batch (crypto/src/lib.rs:206-219) -> nw_verify_batch, one
        2f+1 certificate at 67 / 667 / 6,667 votes (committee cached), and 67 votes with keys
        outside the cache (Pippenger MSM).
    ``keep`` (a dict) receives the inputs of the calls the CPU comparator repeats (cpu_latency)."""
    import numpy as np
    from narwhal_amd import _lib, workload

    def p50(fn, n):
        for _ in range(5):
            fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return {"p50_ms": ts[len(ts) // 2] * 1e3, "p99_ms": ts[int(len(ts) * 0.99)] * 1e3, "min_ms": ts[0] * 1e3,
                "samples": n}

    out = {}
    msg, pk, sig = bytes(cs.msgs[0]), bytes(com.pks[cs.signer[0]]), bytes(cs.sigs[0])
    assert eng.verify_strict(msg, pk, sig)
    out["strict_cached"] = p50(lambda: eng.verify_strict(msg, pk, sig), samples)
    keep = {} if keep is None else keep
    keep["strict"] = (msg, pk, sig)
    keep["certs"] = {}

    def keep_cert(c_com, c_cs, c):
        f, n = int(c_cs.cert_first[c]), int(c_cs.cert_n[c])
        keep["certs"][n] = (bytes(c_cs.msgs[c]), [bytes(c_com.pks[k]) for k in c_cs.signer[f:f + n]],
                            [bytes(x) for x in c_cs.sigs[f:f + n]])

    # n header / vote checks in ONE call (CoreBatcher's batching, core.py): the crossover against n
    # one-at-a-time CPU checks (cpu_latency strict_xN)
    keep["strict_many"] = {}
    for nm in (2, 8, 64):
        sel = [(k * 67) % cs.nsigs for k in range(nm)]
        m_msgs = [bytes(cs.msgs[int(np.searchsorted(cs.cert_first, j, side="right")) - 1]) for j in sel]
        m_pks = [bytes(com.pks[cs.signer[j]]) for j in sel]
        m_sigs = [bytes(cs.sigs[j]) for j in sel]
        mcall = eng.prepare_strict_many_call(m_msgs, m_pks, m_sigs)
        assert all(mcall())
        out["strict_cached_x%d" % nm] = p50(mcall, samples)
        keep["strict_many"][nm] = list(zip(m_msgs, m_pks, m_sigs))
    fseed = np.frombuffer(os.urandom(32), np.uint8).reshape(1, 32)
    fpk, fsig = eng.sign_many_np(fseed, np.frombuffer(msg, np.uint8).reshape(1, 32))
    fpk, fsig = bytes(fpk[0]), bytes(fsig[0])
    assert eng.verify_strict(msg, fpk, fsig)
    out["strict_uncached"] = p50(lambda: eng.verify_strict(msg, fpk, fsig), samples)

    def cert_call(e, c_com, c_cs, c):
        f, n = int(c_cs.cert_first[c]), int(c_cs.cert_n[c])
        m = bytes(c_cs.msgs[c])
        return e.prepare_batch_call([m] * n, [bytes(c_com.pks[k]) for k in c_cs.signer[f:f + n]],
                                    [bytes(x) for x in c_cs.sigs[f:f + n]])

    zseed = os.urandom(32)
    call = cert_call(eng, com, cs, 0)
    assert call(zseed, 0)
    out["batch_cached_%d" % int(cs.cert_n[0])] = p50(lambda: call(zseed, 0), samples)
    keep_cert(com, cs, 0)
    # keys outside the cache: a fresh committee of the same size that is never loaded
    nu = int(cs.cert_n[0])
    useeds = np.frombuffer(os.urandom(32 * nu), np.uint8).reshape(nu, 32).copy()
    ucom = workload.Committee(seeds=useeds, pks=eng.sign_many_np(useeds, np.zeros((nu, 32), np.uint8))[0],
                              stake=np.ones(nu, np.uint32))
    ucs = workload.make_certificates(ucom, 2, ucom.size, eng)
    ucall = cert_call(eng, ucom, ucs, 0)
    assert ucall(zseed, 0)
    out["batch_uncached_%d" % ucom.size] = p50(lambda: ucall(zseed, 0), samples)
    # Header::verify's id check at N = 10,000: one SHA-512 of a 6,667-parent header preimage
    # (author 32 + round 8 + 6,667 x 32 B = 213,384 B, primary/src/messages.rs:50,71-83)
    import hashlib
    pre = os.urandom(32 + 8 + 6667 * 32)
    assert eng.sha512(pre) == hashlib.sha512(pre).digest()
    keep["header"] = pre
    keep["worker_batch"] = workload.worker_batches_np(1)[0].tobytes()
    out["header_digest_6667_parents"] = dict(p50(lambda: eng.sha512(pre), max(20, samples // 4)),
                                             bytes=len(pre),
                                             hashlib_1core_ms=min(timeit_once(lambda: hashlib.sha512(pre).digest())
                                                                  for _ in range(20)) * 1e3)
    for nval in (1000, 10000):
        e2 = _lib.Engine(device=eng.device, key_window=-1)
        c2 = workload.make_committee(nval, e2)
        e2.committee_load_np(c2.pks, c2.stake)
        votes = 2 * nval // 3 + 1
        k_cs = workload.make_certificates(c2, 2, votes, e2)
        kc = cert_call(e2, c2, k_cs, 0)
        keep_cert(c2, k_cs, 0)
        assert kc(zseed, 0)
        out["batch_cached_%d" % votes] = dict(p50(lambda: kc(zseed, 0), max(20, samples // 4)),
                                              key_window=e2.key_window())
        del kc
        e2.close()
    out["note"] = ("host buffers, one ABI call per sample (marshalled once); cached = keys in the committee key "
                   "cache (nw_committee_load at spawn), uncached = variable-base path (k_verify_var / MSM)")
    return out


NW_F_STRICT = 0x008   # include/nwcrypto.h: the verify_strict verdict bit of a signature's flags


def leg_args(args, config, **kw):
    """A copy of ``args`` for another config's leg: that config's own shape (no overrides)."""
    d = dict(vars(args))
    d.update(config=config, validators=None, certs=None, votes=None, streams=None)
    d.update(kw)
    return argparse.Namespace(**d)


class ConfigRun:
    """One BASELINE config's timed step on this rank: engine, committee and
    certificates resident in HBM; the step = nw_verify_certs_dev (+ C4: the rank's worker-batch
    digests on a second stream, worker/src/processor.rs:65) (+ N > 1: the RCCL all-gathers of the
    verdict bitmaps, stake and digests); the warm-up, the timed loop, and the read-back of EVERY
    step's verdicts, accepted stake and input-check status (each step writes its own result set),
    the last step's per-vote flags on every stream and, C4, all digests of the last two steps."""

    def __init__(self, args, world, rank, local):
        import numpy as np
        import torch
        from narwhal_amd import _lib, workload
        t0 = time.perf_counter()
        self.args, self.world, self.rank = args, world, rank
        self.plan = plan = config_plan(args, world, rank)
        self.dev = dev = torch.device("cuda", local)
        self.eng = eng = _lib.Engine(device=local, key_window=args.key_window, flags=args.engine_flags)
        self.com = com = workload.make_committee(plan["validators"], eng)
        self.slots = slots = eng.committee_load_np(com.pks, com.stake)
        self.first_cert = plan["first_cert"]                # each rank: its own shard of certificates
        self.cs = cs = workload.make_certificates(com, plan["ncerts"], plan["votes"], eng, first_cert=self.first_cert)
        self.ranges = plan["ranges"]                        # node-wide certificate ranges
        self.d_sig = torch.from_numpy(cs.sigs).to(dev)
        self.d_signer = torch.from_numpy(slots[cs.signer].astype(np.int32)).to(dev)
        self.d_first = torch.from_numpy(cs.cert_first.astype(np.int32)).to(dev)
        self.d_n = torch.from_numpy(cs.cert_n.astype(np.int32)).to(dev)
        self.d_msg = torch.from_numpy(cs.msgs).to(dev)
        # per-vote flags: one buffer per batch in flight; verdicts / stake / status: one set per step
        self.nst = nst = max(1, args.streams if args.streams is not None else CONFIGS[args.config]["streams"])
        self.flags = [torch.zeros(cs.nsigs, dtype=torch.int32, device=dev) for _ in range(nst)]
        self.streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(nst - 1)]
        self.scratch = self._result_set()
        self.res = []
        self.zseed = os.urandom(32)
        # C4: the rank's worker-batch digests run inside the timed step on a second stream,
        # concurrently with the verify kernels; the step ends when both are done
        self.ndig = ndig = plan["digest_batches"]
        self.from_host = bool(ndig) and args.batches == "host"
        self.pipelined = bool(ndig) and not args.digest_join
        if ndig:
            self.host_b = workload.worker_batches_np(ndig)
            self.blen = blen = self.host_b.shape[1]
            self.d_boff = torch.arange(ndig, dtype=torch.int64, device=dev) * blen
            self.d_blen = torch.full((ndig,), blen, dtype=torch.int64, device=dev)
            # joined: one digest stream per batch in flight.  Pipelined: two alternating digest streams
            # at high priority (step i + 1's digests run beside the tail of step i's), each with its
            # output and, with host batches, its upload buffer (step i's batches are DMA'd on step i's
            # digest stream)
            ndst = 2 if self.pipelined else nst
            self.d_bouts = [torch.empty((ndig, 64), dtype=torch.uint8, device=dev) for _ in range(ndst)]
            self.s_digs = [torch.cuda.Stream(device=dev, priority=-1 if self.pipelined else 0) for _ in range(ndst)]
            self.ev_digs = [torch.cuda.Event() for _ in range(ndst)]
            if self.from_host:
                self.uploader = BatchUploader(self.host_b, dev, nbuf=2,
                                              copy_streams=self.s_digs if self.pipelined else None)
                self.d_bdata = None
            else:
                self.d_bdata = torch.from_numpy(self.host_b.reshape(-1)).to(dev)
        # N > 1: every all_gather on one stream (collectives of one communicator stay serialized),
        # after its batch's kernels
        self.s_comm = torch.cuda.Stream(device=dev) if world > 1 and nst > 1 else None
        self.n_step = 0
        self.ev_pre = None
        torch.cuda.synchronize()       # inputs resident before any stream reads them
        self.setup_s = time.perf_counter() - t0

    def _result_set(self):
        import torch
        n = self.cs.ncerts
        return (torch.zeros(n, dtype=torch.uint8, device=self.dev), torch.zeros(n, dtype=torch.int64, device=self.dev),
                torch.zeros(1, dtype=torch.int32, device=self.dev))

    def verify_step(self, stream, flags=None, res=None):
        cs = self.cs
        ok, stake, status = self.scratch if res is None else res
        flags = self.flags[0] if flags is None else flags
        self.eng.verify_certs_dev(cs.ncerts, self.d_first.data_ptr(), self.d_n.data_ptr(), cs.nsigs,
                                  self.d_sig.data_ptr(), self.d_signer.data_ptr(), self.d_msg.data_ptr(), self.zseed,
                                  self.first_cert, ok.data_ptr(), flags.data_ptr(), stake.data_ptr(),
                                  stream.cuda_stream, d_status=status.data_ptr())

    def step(self):
        from narwhal_amd import shard
        import torch
        i = self.n_step
        self.n_step += 1
        cur, flags = self.streams[i % self.nst], self.flags[i % self.nst]
        res = self.res[i] if i < len(self.res) else self.scratch
        ndig, s_dig = self.ndig, None
        if ndig:
            # launched before the step's verify kernels, so the digest workgroups get their (exclusive)
            # CUs first; the step ends when both are done.  (Not joining the streams per step, so
            # that step i + 1's digests start while step i verifies, measured slower: 414-437 vs
            # 486-491 M sigs/s, r04r: a digest launched while k_verify holds every CU waits for CUs;
            # two alternating digest streams without the join, 460 M, r04u: the second stream's digest
            # still started only when the first finished, then waited for CUs.)
            di = i % len(self.s_digs)
            s_dig, ev_dig = self.s_digs[di], self.ev_digs[di]
            # Joined: after the previous step's verify kernels (a digest enqueued while k_verify holds
            # every CU waits for whole CUs to drain: its workgroups take a CU each).  Pipelined: only
            # after its own stream's earlier work (step i-2's digests, this step's upload), so it is
            # queued while step i-1's k_verify still runs and takes CUs as that grid's dispatch ends,
            # ahead of step i's k_verify (which waits for step i-1's k_finish); when both became ready
            # at the same event, the verify grid won the CUs in about one run in three and the digests
            # ran 26.7 instead of 16-17 ms (profiles/r05/c4_hwq_r05.txt)
            if not self.pipelined:
                s_dig.wait_stream(cur)
            elif self.ev_pre is not None:
                s_dig.wait_event(self.ev_pre)   # no earlier than step i-1's verify kernels (HBM batches
                #                                 would otherwise let the digest streams run steps ahead)
            src = self.uploader.ready_buffer(s_dig) if self.from_host else self.d_bdata
            self.eng.sha512_many_dev(src.data_ptr(), self.d_boff.data_ptr(), self.d_blen.data_ptr(), ndig,
                                     self.d_bouts[di].data_ptr(), s_dig.cuda_stream)
            ev_dig.record(s_dig)
        if self.pipelined:
            self.ev_pre = torch.cuda.Event()
            self.ev_pre.record(cur)             # this step's verify kernels start here
        self.verify_step(cur, flags, res)
        if self.from_host:
            # host threads stage the NEXT step's batches into pinned memory and DMA them while this
            # step's kernels run (the next step's digests wait for that upload; the timed region's
            # closing synchronize waits for every upload)
            self.uploader.stage_next(read_stream=s_dig)
        if ndig and not self.pipelined:
            cur.wait_event(ev_dig)
        if self.world > 1:
            # RCCL all_gathers of the verdict bitmaps + stake and (C4) of the ranks' worker digests
            # (32 B per batch), after this step's kernels.  Pipelined: the digests all-gathered in
            # step i are step i - 1's (finished while step i verified); the last step's after the loop
            dig_out = None
            if ndig and not self.pipelined:
                dig_out = self.d_bouts[i % len(self.d_bouts)]
            elif ndig and i > 0:
                dig_out = self.d_bouts[(i - 1) % len(self.d_bouts)]
                cur.wait_event(self.ev_digs[(i - 1) % len(self.ev_digs)])
            if self.s_comm is None:
                if dig_out is not None:
                    shard.allgather_digests(dig_out)
                shard.allgather_verdicts(res[0], res[1], self.ranges)
            else:
                self.s_comm.wait_stream(cur)
                with torch.cuda.stream(self.s_comm):
                    if dig_out is not None:
                        shard.allgather_digests(dig_out)
                    shard.allgather_verdicts(res[0], res[1], self.ranges)
                cur.wait_stream(self.s_comm)

    def drain_digests(self):
        """Pipelined C4: the last step's digests (and, N > 1, their all-gather) inside the timed region."""
        from narwhal_amd import shard
        if not self.pipelined or self.n_step == 0:
            return
        i = self.n_step - 1
        cur = self.streams[i % self.nst]
        cur.wait_event(self.ev_digs[i % len(self.ev_digs)])
        if self.world > 1:
            shard.allgather_digests(self.d_bouts[i % len(self.d_bouts)])

    def run(self, steps, warmup):
        """W untimed warm-up steps, then EXACTLY ``steps`` steps bracketed by a barrier and a
        synchronize on both sides; returns (max-over-ranks seconds, output checks)."""
        import torch
        import torch.distributed as dist
        self.res = [self._result_set() for _ in range(warmup + steps)]
        if self.from_host:
            self.uploader.stage_next(read_stream=None)   # the first step's batches
        torch.cuda.synchronize()
        for _ in range(warmup):
            self.step()
        if self.ndig:
            self.drain_digests()
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        self.eng.profile_read()             # discard warm-up events
        self.eng.profile_enable(True)
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        if self.ndig:
            self.drain_digests()
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        self.eng.profile_enable(False)
        self.prof = self.eng.profile_read()
        checks = self.check_outputs(warmup, steps)
        if self.world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            okt = torch.tensor([1 if checks["ok"] else 0], dtype=torch.int32, device=self.dev)
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
            checks["ok_all_ranks"] = bool(okt.item())
        self.steps, self.warmup, self.elapsed = steps, warmup, elapsed
        return elapsed, checks

    def expected_digests(self):
        """hashlib SHA-512 of this rank's worker batches (threads: hashlib releases the GIL)."""
        import hashlib
        import numpy as np
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(8) as ex:
            ds = list(ex.map(lambda b: hashlib.sha512(b.data).digest(), self.host_b))
        return np.frombuffer(b"".join(ds), np.uint8).reshape(len(ds), 64)

    def check_outputs(self, warmup, steps):
        """Every step's certificate verdicts, accepted stake and input-check status (the committee is
        honest with stake 1 per key, so each certificate's accepted stake is its vote count), the
        last step's per-vote flags on each stream (strict bit set), and C4's digests."""
        import numpy as np
        votes = self.plan["votes"]
        bad = []
        for k, (ok, stake, st) in enumerate(self.res):
            if not (bool(ok.all().item()) and bool((stake == votes).all().item()) and int(st.item()) == 0):
                bad.append(k)
        used = min(self.nst, warmup + steps)
        strict = all(bool(((f & NW_F_STRICT) != 0).all().item()) for f in self.flags[:used])
        out = {"steps_checked": warmup + steps, "timed_steps_checked": steps, "bad_steps": bad,
               "last_flags_all_strict": strict,
               "what": "every step's %d certificate verdicts + accepted stake + status word (own result set per "
                       "step), and the %d per-vote flags of the last step on each of %d stream(s)"
                       % (self.cs.ncerts, self.cs.nsigs, used)}
        dig_ok = True
        if self.ndig:
            exp = self.expected_digests()
            nb = min(len(self.d_bouts), warmup + steps)
            dig_ok = all(np.array_equal(d.cpu().numpy(), exp) for d in self.d_bouts[:nb])
            out["digests_ok"] = dig_ok
            out["digests_what"] = ("all %d digests written by the last %d step(s) vs hashlib SHA-512 of the batches"
                                   % (self.ndig, nb))
        out["ok"] = not bad and strict and dig_ok
        return out

    def isolated(self, launches=3):
        """k_verify launched alone after the timed region, the GPU idle between launches."""
        import torch
        self.eng.profile_enable(True)
        for _ in range(launches):
            self.verify_step(self.streams[0])
            torch.cuda.synchronize()
        self.eng.profile_enable(False)
        return self.eng.profile_read()

    def roofline(self, iso, with_profiles):
        """k_verify's fraction of the measured MAD peak (work model: kverify_fm_per_sig)."""
        kms, kn, ksigs = self.prof
        avg_launch_s = (kms / kn) / 1e3 if kn else float("nan")
        if ksigs is None:                              # library without nw_profile_read_sigs (A/B runs)
            ksigs = self.cs.nsigs * kn
        sigs_per_launch = ksigs / kn if kn else 0.0
        kw = self.eng.key_window()
        bw = self.eng.base_window()
        fm = kverify_fm_per_sig(kw, bw)
        peak = valu_peak_mad_per_s() / 1e12
        achieved = sigs_per_launch * fm * MADS_PER_FM / avg_launch_s / 1e12
        v1 = COST_MODEL_V1_FM.get(self.plan["votes"])
        nst = self.nst
        return {
            "bound": "valu", "kernel": "k_verify", "achieved": achieved, "peak": peak, "unit": "TMAD/s",
            "frac": achieved / peak,
            "traffic": traffic_per_launch() if with_profiles else None,
            "per_cycle": clock_frac_profile() if with_profiles else None,
            "avg_launch_ms": avg_launch_s * 1e3, "launches": kn,
            "batches_in_flight": nst,
            "isolated": None if not iso or not iso[1] else {
                "avg_launch_ms": iso[0] / iso[1], "launches": iso[1],
                "frac": sigs_per_launch * fm * MADS_PER_FM / (iso[0] / iso[1] / 1e3) / 1e12 / peak,
                "note": "k_verify launched alone after the timed region, the GPU idle between launches (frac "
                        "above: the timed launches, back to back%s)" % (
                            ", overlapping the other batch's kernels" if nst > 1 else "")},
            "work_model": "%.0f sigs/launch (%d launches per step) x %d FM/sig (7 FM per mixed addition x (%d basepoint "
                          "+ %d key - 1) comb positions + 1 FM for the chain's first entry - 1 FM (no T in the last "
                          "addition), key window %d) x 100 u32 MADs; SHA-512/mod-l/recoding VALU work not counted; "
                          "peak = measured v_mad_u64_u32 rate"
                          % (sigs_per_launch, kn // max(1, self.steps), fm, comb_pos(bw), comb_pos(kw), kw),
            "dalek_equiv": {"fm_per_sig": v1, "TMADps": (sigs_per_launch * v1 * MADS_PER_FM / avg_launch_s / 1e12)
                            if v1 else None,
                            "note": "SURVEY §8(d) cost model v1 = dalek's MSM work per signature; the comb "
                                    "algorithm needs %.1fx fewer FM" % (v1 / fm) if v1 else ""},
        }

    def workload_desc(self):
        plan, cs = self.plan, self.cs
        strong = plan["scaling"] == "strong"
        desc = ("%s: %d-validator committee, %d certificates x %d votes (%d sigs) %s"
                % (self.args.config, plan["validators"], plan["node_certs"] if strong else plan["ncerts"],
                   plan["votes"], plan["total_sigs"] if strong else cs.nsigs,
                   "per node round, partitioned over the GPUs" if strong else "per GPU"))
        if self.ndig:
            desc += " + %d worker-batch SHA-512 digests (%d B each) per GPU on a second stream" % (self.ndig, self.blen)
            if self.from_host:
                desc += (", batches from pageable host memory (staged to pinned + H2D inside the timed loop, "
                         "double-buffered)")
        return desc

    def digest_in_step(self):
        if not self.ndig:
            return None
        d = {"batches_per_gpu": self.ndig, "bytes_per_gpu_per_step": self.ndig * self.blen,
             "GBps_per_gpu": self.ndig * self.blen * self.steps / self.elapsed / 1e9,
             "batches_from_host": self.from_host}
        if self.from_host:
            d["upload"] = self.uploader.stats()
        return d

    def close(self):
        """Release the engine (its key tables) and this run's device buffers."""
        import torch
        torch.cuda.synchronize()
        self.eng.close()
        for k in ("d_sig", "d_signer", "d_first", "d_n", "d_msg", "flags", "scratch", "res", "d_boff", "d_blen",
                  "d_bouts", "d_bdata", "uploader"):
            if hasattr(self, k):
                setattr(self, k, None)
        torch.cuda.empty_cache()


def cert_latency(run, samples):
    """Single-certificate latency through nw_verify_certs from host buffers (H2D -> kernels -> D2H),
    the Core::run usage pattern; p50 / p99 over ``samples`` calls."""
    import numpy as np
    cs, lat = run.cs, []
    for i in range(samples):
        c = i % cs.ncerts
        f, n = int(cs.cert_first[c]), int(cs.cert_n[c])
        t1 = time.perf_counter()
        cok, _, _ = run.eng.verify_certs_np(np.array([0], np.uint32), np.array([n], np.uint32), cs.sigs[f:f + n],
                                            run.slots[cs.signer[f:f + n]], cs.msgs[c:c + 1], run.zseed,
                                            run.first_cert + c)
        lat.append(time.perf_counter() - t1)
        assert cok[0] == 1
    lat.sort()
    return (lat[len(lat) // 2] * 1e3, lat[int(len(lat) * 0.99)] * 1e3) if lat else (None, None)


def c4_block(run, elapsed, checks, iso):
    """The north-star config's leg (configs[3]): one GPU's share of a 10,000-validator node round."""
    plan = run.plan
    total = plan["total_sigs"] * run.steps
    kw = run.eng.key_window()
    return {"config": run.workload_desc(), "baseline_config": plan["baseline"],
            "value": total / elapsed, "unit": "sigs/s", "n_gpus": run.world, "steps": run.steps,
            "warmup": run.warmup, "ms_per_step": elapsed / run.steps * 1e3, "scaling": plan["scaling"],
            "key_window": kw, "key_negtab": run.eng.key_negtab(),
            "kverify_fm_per_sig": kverify_fm_per_sig(kw, run.eng.base_window()),
            "roofline": run.roofline(iso, False), "digest_in_step": run.digest_in_step(),
            "checks": checks, "setup_s": run.setup_s}


def cpu_latency(inp, gpu, samples=100):
    """One-call latencies on ONE host thread, the reference's usage: Core verifies each header / vote
    inline (primary/src/core.rs:306-346) with crypto::Signature::verify -> dalek verify_strict, each
    certificate with Signature::verify_batch (crypto/src/lib.rs:200-219), and the worker hashes each
    batch with SHA-512 (worker/src/processor.rs:65).  oracle/nw_ref.c is the C restatement of dalek
    1.0.1 (strict: its double-base NAF5/NAF8 with the precomputed basepoint table; certificates:
    per-vote key decompression + Straus below 190 points, Pippenger above); hashlib (OpenSSL) for the
    digests.  Same inputs as the GPU calls; ``cpu_over_gpu`` > 1 means the GPU call is faster."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import nw_ref   # test/baseline only

    def stats(fn, n):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return {"p50_ms": ts[len(ts) // 2] * 1e3, "p99_ms": ts[min(n - 1, int(n * 0.99))] * 1e3,
                "min_ms": ts[0] * 1e3, "samples": n}

    out = {}
    msg, pk, sig = inp["strict"]
    assert nw_ref.verify_strict(pk, msg, sig)
    out["strict"] = stats(lambda: nw_ref.verify_strict(pk, msg, sig), 2 * samples)
    for nm, triples in sorted(inp.get("strict_many", {}).items()):
        assert all(nw_ref.verify_strict(p_, m_, s_) for m_, p_, s_ in triples)
        out["strict_x%d" % nm] = stats(lambda: [nw_ref.verify_strict(p_, m_, s_) for m_, p_, s_ in triples],
                                       max(20, samples // max(1, nm // 8)))
    zseed = bytes(32)
    for votes, (digest, pks, sigs) in sorted(inp["certs"].items()):
        call = nw_ref.prepare_crypto_verify_batch(digest, pks, sigs)
        assert call(zseed, 0)
        out["cert_%d" % votes] = stats(lambda: call(zseed, 0), samples)
    batch = inp["worker_batch"]
    out["worker_batch"] = dict(stats(lambda: hashlib.sha512(batch).digest(), samples), bytes=len(batch))
    pre = inp["header"]
    out["header_6667_parents"] = dict(stats(lambda: hashlib.sha512(pre).digest(), samples), bytes=len(pre))
    for k, g in gpu.items():
        if k in out and g:
            out[k]["gpu_p50_ms"] = g[0]
            out[k]["gpu_source"] = g[1]
            out[k]["cpu_over_gpu"] = out[k]["p50_ms"] / g[0]
    out["threads"] = 1
    out["cpu_model"] = cpu_model()
    out["note"] = ("one host thread, one call at a time (no batching across calls), p50/p99 over the samples; "
                   "cpu_over_gpu = CPU p50 / GPU p50 of the same call on the same inputs (> 1: the GPU is faster)")
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.hw_queues:
        # HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES in-order hardware queues (4 by
        # default).  Left at 4: with 16 a C2 step ran 3.1 instead of 1.36 ms (stalls of ~14 ms between
        # steps, the GPU idle) and C4 434 instead of 575 M sigs/s (profiles/r05/c4_hwq_r05.txt); the
        # C4 step instead keeps each upload on the stream of the digests that read it.
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    if args.dry_run:
        return dry_run(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world), file=sys.stderr)
    torch.cuda.set_device(local)
    gloo_group = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        gloo_group = dist.new_group(backend="gloo")   # host-side barrier for the CPU-baseline leg

    from narwhal_amd import _lib, workload
    run = ConfigRun(args, world, rank, local)
    plan = run.plan
    elapsed, checks = run.run(args.steps, args.warmup)
    if not args.timing_only:
        assert checks.get("ok_all_ranks", checks["ok"]), "honest workload rejected (or a digest mismatched): %r" % checks
    total_sigs = plan["total_sigs"] * args.steps       # every rank's signatures (node-wide)
    value = total_sigs / elapsed

    out = None
    c2 = args.config == "C2"
    cpu_inp = {}
    if rank == 0:
        iso = run.isolated()
        roofline = run.roofline(iso, c2)
        p50c, p99c = cert_latency(run, args.latency_samples)
        out = {
            "metric": METRIC, "value": value, "unit": "sigs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": plan["scaling"], "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (GPU-signed RFC 8032 signatures over SHA-512 certificate digests)",
            "config": {"workload": run.workload_desc(), "baseline_config": plan["baseline"],
                       "validators": plan["validators"], "certs_per_gpu": run.cs.ncerts,
                       "votes_per_cert": plan["votes"], "key_window": run.eng.key_window(),
                       "key_negtab": run.eng.key_negtab(),
                       "parallelism": "certificate shards per GPU; RCCL all_gather of verdict bitmaps + stake"},
            "p50_cert_latency_ms": p50c, "p99_cert_latency_ms": p99c,
            "roofline": roofline, "checks": checks, "build": _lib.version(),
        }
        if run.ndig:
            out["digest_in_step"] = run.digest_in_step()
        # GPU legs first: the CPU baselines run more threads than the container's CPU quota, and the
        # cgroup throttling that follows would slow the host side of the next leg
        if world == 1 and c2 and not args.no_extras:
            out["host_fed"] = host_fed(run.eng, run.cs, run.slots, run.zseed)
            out["msm"] = msm_leg(run.eng)
            out["worker_digest"] = worker_digest_leg(run.eng)
            if args.latency_samples > 0:
                out["latency"] = latency_legs(run.eng, run.com, run.slots, run.cs, args.latency_samples, keep=cpu_inp)
        if world == 1 and c2 and args.digest_batches > 0:
            out["digest"] = digest_leg(run.eng, run.dev, args.digest_batches, args.digest_share, 3, 0.0,
                                       run.verify_step)
    # the north-star config (configs[3]) in the same run, after the C2 engine is closed: one GPU's
    # share of a 10,000-validator node round (1,250 certificates x 6,667 votes + 1,250 host-resident
    # worker batches), at every world size
    c4run = None
    if c2 and args.c4_steps > 0:
        run.close()
        c4run = ConfigRun(leg_args(args, "C4"), world, rank, local)
        el4, ch4 = c4run.run(args.c4_steps, args.c4_warmup)
        if not args.timing_only:
            assert ch4.get("ok_all_ranks", ch4["ok"]), "C4 leg: honest workload rejected or digest mismatch: %r" % ch4
        if rank == 0:
            out["c4"] = c4_block(c4run, el4, ch4, c4run.isolated())
    if rank == 0:
        if not args.no_cpu_baseline:
            # every line carries the host baseline, N > 1 included: rank 0 times it after the timed
            # region while the other ranks block in a gloo barrier (a socket wait, no spinning host
            # thread to steal the cores being measured)
            cb = cpu_baseline(run.cs, run.com, args.cpu_seconds, label=args.config)
            if run.ndig:
                cb["with_digests"] = cpu_step_with_digests(cb, run.host_b, plan, args.cpu_seconds / 3)
            cb["gpu_over_cpu"] = value / cb["value"]          # against the measured slice
            cb["gpu_over_host_extrapolated"] = value / cb["host_extrapolated"]["value"]   # against the whole host
            cb["ratios_note"] = ("gpu_over_cpu: this run's %d GPU(s) vs the measured %.0f-CPU slice; "
                                 "gpu_over_host_extrapolated: vs the whole host's %d physical cores (north star: "
                                 ">= 50x the host at 8 GPUs)" % (world, cb["measured_slice"]["cpus"],
                                                                  cb["host_extrapolated"]["physical_cores"]))
            if run.ndig:
                cb["with_digests"]["gpu_over_cpu"] = value / cb["with_digests"]["sigs_per_s"]
            if cpu_inp:
                lat = out["latency"]
                wd = out.get("worker_digest", {}).get("one_batch_call_ms", {})
                gpu = {"strict": (lat["strict_cached"]["p50_ms"], "latency.strict_cached"),
                       **{"strict_x%d" % nm: (lat["strict_cached_x%d" % nm]["p50_ms"], "latency.strict_cached_x%d" % nm)
                          for nm in (2, 8, 64) if "strict_cached_x%d" % nm in lat},
                       "cert_67": (p50c, "p50_cert_latency_ms (nw_verify_certs, one C2 certificate)"),
                       "cert_667": (lat["batch_cached_667"]["p50_ms"], "latency.batch_cached_667"),
                       "cert_6667": (lat["batch_cached_6667"]["p50_ms"], "latency.batch_cached_6667"),
                       "worker_batch": (wd.get("p50"), "worker_digest.one_batch_call_ms"),
                       "header_6667_parents": (lat["header_digest_6667_parents"]["p50_ms"],
                                               "latency.header_digest_6667_parents")}
                cb["latency"] = cpu_latency(cpu_inp, gpu, args.cpu_latency_samples)
                out["p50_cert_latency_cpu_ms"] = cb["latency"]["cert_67"]["p50_ms"]
            out["cpu_baseline"] = cb
            if "digest" in out:
                hb = c4run.host_b if c4run is not None else workload.worker_batches_np(256)
                threads = max(cpu_thread_candidates())
                bps, nb, dt = hashlib_rate(hb, threads, 3.0)
                out["digest"]["cpu_baseline"] = {"GBps": bps / 1e9, "cores": threads,
                                                 "kind": "hashlib (OpenSSL) SHA-512",
                                                 "per_gpu_share_GBps": bps / 1e9 / GPUS_PER_NODE,
                                                 "sample": "%d batches in %.1f s on %d threads" % (nb, dt, threads)}
            if c4run is not None:
                c4 = out["c4"]
                threads = cb["measured_slice"]["threads"]
                c4cb = cpu_baseline(c4run.cs, c4run.com, args.cpu_seconds / 2, label="C4", threads=threads)
                c4cb["with_digests"] = cpu_step_with_digests(c4cb, c4run.host_b, c4run.plan, args.cpu_seconds / 5)
                c4cb["gpu_over_cpu"] = c4["value"] / c4cb["with_digests"]["sigs_per_s"]
                c4cb["gpu_over_host_extrapolated"] = c4["value"] / (
                    c4cb["host_extrapolated"]["value"] * c4cb["with_digests"]["sigs_per_s"] / c4cb["value"])
                c4cb["ratios_note"] = ("C4 step (verify + worker digests) on %d GPU(s) vs the same step done by the "
                                       "measured %.0f-CPU slice (gpu_over_cpu) and by the whole host extrapolated "
                                       "to its physical cores (north star: >= 50x the host at 8 GPUs)"
                                       % (world, c4cb["measured_slice"]["cpus"]))
                c4["cpu_baseline"] = c4cb
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier(group=gloo_group)    # ranks > 0 wait here while rank 0 times the host baseline
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
