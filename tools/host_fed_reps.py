"""host_fed outliers: the bench's host_fed leg repeated, with every call's
start / end on the host clock, so a slow pass can be attributed to the calls (and threads) that
made it slow.  Usage (GPU box): python tools/host_fed_reps.py PASSES > gpurun_out/host_fed_reps.json
Optional second argument "trace": one marker print per pass for a rocprofv3 timeline."""
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    no_gc = "nogc" in sys.argv[2:]   # Python's cyclic GC off during the timed passes
    from narwhal_amd import _lib, workload
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0, key_window=-1)
    com = workload.make_committee(100, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, 14926, 67, eng)
    zseed = os.urandom(32)
    chunks, threads = 8, 4
    bounds = np.linspace(0, cs.ncerts, chunks + 1).astype(int)
    parts = []
    for a, b in zip(bounds, bounds[1:]):
        f0, f1 = int(cs.cert_first[a]), int(cs.cert_first[b - 1] + cs.cert_n[b - 1])
        parts.append((cs.cert_first[a:b] - f0, cs.cert_n[a:b], np.ascontiguousarray(cs.sigs[f0:f1]),
                      np.ascontiguousarray(slots[cs.signer[f0:f1]]), np.ascontiguousarray(cs.msgs[a:b]), int(a)))
    def cpu_stat():
        try:
            with open("/sys/fs/cgroup/cpu.stat") as f:
                return {k: int(v) for k, v in (line.split() for line in f)}
        except (OSError, ValueError):
            return {}

    log = []
    lock = threading.Lock()
    st0 = cpu_stat()
    t_origin = time.perf_counter()

    def run(k, p, rep):
        t0 = time.perf_counter()
        ok, _, _ = eng.verify_certs_np(p[0], p[1], p[2], p[3], p[4], zseed, p[5])
        t1 = time.perf_counter()
        with lock:
            log.append({"pass": rep, "call": k, "thread": threading.get_ident() % 10007,
                        "start_ms": (t0 - t_origin) * 1e3, "ms": (t1 - t0) * 1e3})
        return bool(ok.all())

    out = {"passes": [], "gc_disabled": no_gc}
    import gc
    gc.collect()
    if no_gc:
        gc.disable()
    with ThreadPoolExecutor(threads) as ex:
        assert all(ex.map(lambda kp: run(kp[0], kp[1], -1), enumerate(parts)))
        for rep in range(passes):
            t0 = time.perf_counter()
            ok = all(ex.map(lambda kp: run(kp[0], kp[1], rep), enumerate(parts)))
            dt = time.perf_counter() - t0
            assert ok
            out["passes"].append({"pass": rep, "ms": dt * 1e3, "start_ms": (t0 - t_origin) * 1e3})
        # the same calls on newly allocated host arrays every pass (a node's network buffers)
        out["fresh_passes_ms"] = []
        for rep in range(min(passes, 8)):
            fr = [(a, b, c.copy(), d.copy(), e.copy(), f) for a, b, c, d, e, f in parts]
            t0 = time.perf_counter()
            ok = all(ex.map(lambda kp: run(kp[0], kp[1], 1000 + rep), enumerate(fr)))
            out["fresh_passes_ms"].append((time.perf_counter() - t0) * 1e3)
            assert ok
    ms = sorted(p["ms"] for p in out["passes"])
    med = ms[len(ms) // 2]
    out["median_ms"] = med
    out["slow_passes"] = [p for p in out["passes"] if p["ms"] > 1.3 * med]
    slow_ids = {p["pass"] for p in out["slow_passes"]}
    out["calls_of_slow_passes"] = [c for c in log if c["pass"] in slow_ids]
    cm = sorted(c["ms"] for c in log if c["pass"] >= 0)
    out["call_ms_median"] = cm[len(cm) // 2]
    out["call_ms_max"] = cm[-1]
    st1 = cpu_stat()
    out["cgroup_cpu_stat_delta"] = {k: st1[k] - st0.get(k, 0) for k in st1}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
