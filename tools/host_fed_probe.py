"""Where the host-buffer certificate path spends its time (GPU box): host memcpy bandwidth into
pinned memory, pinned H2D bandwidth, and nw_verify_certs on C2 host buffers split into calls over
threads.  Prints one JSON object.  Usage: python tools/host_fed_probe.py > gpurun_out/host_fed.json"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before libnwcrypto: shared HIP runtime)


def best(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    from narwhal_amd import _lib, workload
    out = {}
    nbytes = 68 << 20
    src = np.frombuffer(os.urandom(nbytes), np.uint8).copy()
    pinned = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    pn = pinned.numpy()
    dt = best(lambda: np.copyto(pn, src))
    out["memcpy_to_pinned_GBps_1thread"] = nbytes / dt / 1e9
    dev = torch.device("cuda", 0)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)

    def h2d():
        d.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
    out["h2d_pinned_GBps"] = nbytes / best(h2d) / 1e9
    srct = torch.from_numpy(src)

    def h2d_pageable():
        d.copy_(srct)
        torch.cuda.synchronize()
    out["h2d_pageable_GBps"] = nbytes / best(h2d_pageable) / 1e9

    eng = _lib.Engine(device=0, key_window=-1)
    com = workload.make_committee(100, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, 14926, 67, eng)
    zseed = os.urandom(32)

    def parts(chunks):
        bounds = np.linspace(0, cs.ncerts, chunks + 1).astype(int)
        ps = []
        for a, b in zip(bounds, bounds[1:]):
            f0, f1 = int(cs.cert_first[a]), int(cs.cert_first[b - 1] + cs.cert_n[b - 1])
            ps.append((cs.cert_first[a:b] - f0, cs.cert_n[a:b], np.ascontiguousarray(cs.sigs[f0:f1]),
                       np.ascontiguousarray(slots[cs.signer[f0:f1]]), np.ascontiguousarray(cs.msgs[a:b]), int(a)))
        return ps

    def run(p):
        ok, _, _ = eng.verify_certs_np(p[0], p[1], p[2], p[3], p[4], zseed, p[5])
        assert ok.all()

    res = {}
    for chunks, threads in ((1, 1), (8, 1), (8, 4), (8, 8), (16, 8), (32, 16)):
        ps = parts(chunks)
        with ThreadPoolExecutor(threads) as ex:
            def go():
                list(ex.map(run, ps))
            dt = best(go, reps=3)
        res["%d calls / %d threads" % (chunks, threads)] = {"ms": dt * 1e3, "Msigs_per_s": cs.nsigs / dt / 1e6}
        print(chunks, threads, dt * 1e3, file=sys.stderr, flush=True)
    out["verify_certs_host"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
