"""host_fed shapes: C2 (1,000,042 signatures) from pageable host buffers through
nw_verify_certs, cut into CALLS calls on THREADS host threads, median pass time of REPS passes.

    python3 tools/host_fed_sweep.py [CALLSxTHREADS ...]     (default 8x4 8x8 16x8 4x4 2x2)

One JSON line per shape: pass ms (median, max), M sigs/s, per-call host ms (median)."""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    shapes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]] or [(8, 4), (8, 8), (16, 8), (4, 4), (2, 2)]
    from narwhal_amd import _lib, workload
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0, key_window=-1)
    com = workload.make_committee(100, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, 14926, 67, eng)
    zseed = os.urandom(32)
    for calls, threads in shapes:
        bounds = np.linspace(0, cs.ncerts, calls + 1).astype(int)
        parts = []
        for a, b in zip(bounds, bounds[1:]):
            f0, f1 = int(cs.cert_first[a]), int(cs.cert_first[b - 1] + cs.cert_n[b - 1])
            parts.append((cs.cert_first[a:b] - f0, cs.cert_n[a:b], np.ascontiguousarray(cs.sigs[f0:f1]),
                          np.ascontiguousarray(slots[cs.signer[f0:f1]]), np.ascontiguousarray(cs.msgs[a:b]), int(a)))
        call_ms = []

        def run(p):
            t0 = time.perf_counter()
            ok, _, _ = eng.verify_certs_np(p[0], p[1], p[2], p[3], p[4], zseed, p[5])
            call_ms.append((time.perf_counter() - t0) * 1e3)
            return bool(ok.all())

        with ThreadPoolExecutor(threads) as ex:
            for _ in range(2):
                assert all(ex.map(run, parts))
            call_ms.clear()
            ts = []
            for _ in range(9):
                t0 = time.perf_counter()
                assert all(ex.map(run, parts))
                ts.append((time.perf_counter() - t0) * 1e3)
            # streaming: 9 passes' worth of calls back to back on the same threads, no barrier per pass
            t0 = time.perf_counter()
            assert all(ex.map(run, parts * 9))
            t_stream = (time.perf_counter() - t0) * 1e3
        ts.sort()
        call_ms.sort()
        print(json.dumps({"calls": calls, "threads": threads, "pass_ms_p50": ts[len(ts) // 2], "pass_ms_max": ts[-1],
                          "pass_ms_all": [round(t, 2) for t in ts],
                          "Msigs_per_s": cs.nsigs / ts[len(ts) // 2] / 1e3,
                          "stream_Msigs_per_s": 9 * cs.nsigs / t_stream / 1e3,
                          "call_ms_p50": call_ms[len(call_ms) // 2]}), flush=True)


if __name__ == "__main__":
    main()
