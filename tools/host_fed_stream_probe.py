"""host_fed streaming probe: C2 from pageable host buffers, 16 calls x 8 threads, 20 passes' calls
back to back, in three orders: reused arrays, 4 rotating fresh sets (bench.py's host_fed value), and
the fresh sets again once everything is warm.  Per mode: M sigs/s and the slowest call.

    python3 tools/host_fed_stream_probe.py [rounds]
"""
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from narwhal_amd import _lib, workload
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0, key_window=-1)
    com = workload.make_committee(100, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, 14926, 67, eng)
    zseed = os.urandom(32)
    bounds = np.linspace(0, cs.ncerts, 17).astype(int)
    parts = []
    for a, b in zip(bounds, bounds[1:]):
        f0, f1 = int(cs.cert_first[a]), int(cs.cert_first[b - 1] + cs.cert_n[b - 1])
        parts.append((cs.cert_first[a:b] - f0, cs.cert_n[a:b], np.ascontiguousarray(cs.sigs[f0:f1]),
                      np.ascontiguousarray(slots[cs.signer[f0:f1]]), np.ascontiguousarray(cs.msgs[a:b]), int(a)))
    fresh = [[(a, b, c.copy(), d.copy(), e.copy(), f) for a, b, c, d, e, f in parts] for _ in range(4)]
    call_ms = []

    def run(p):
        t0 = time.perf_counter()
        ok, _, _ = eng.verify_certs_np(p[0], p[1], p[2], p[3], p[4], zseed, p[5])
        call_ms.append((time.perf_counter() - t0) * 1e3)
        return bool(ok.all())

    with ThreadPoolExecutor(8) as ex:
        assert all(ex.map(run, parts))
        for r in range(rounds):
            for mode in ("fresh_sets", "reused", "fresh_sets_warm"):
                calls = parts * 20 if mode == "reused" else [p for k in range(20) for p in fresh[k % 4]]
                call_ms.clear()
                t0 = time.perf_counter()
                assert all(ex.map(run, calls))
                dt = time.perf_counter() - t0
                call_ms.sort()
                print(json.dumps({"round": r, "mode": mode, "Msigs_per_s": round(20 * cs.nsigs / dt / 1e6, 1),
                                  "ms_per_pass": round(dt / 20 * 1e3, 3), "call_ms_p50": round(call_ms[len(call_ms) // 2], 3),
                                  "call_ms_max": round(call_ms[-1], 3),
                                  "calls_over_5ms": sum(1 for c in call_ms if c > 5.0)}), flush=True)


if __name__ == "__main__":
    main()
