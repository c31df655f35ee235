"""Single-certificate latency (the Core::run pattern: one 2f+1 certificate per nw_verify_certs call,
host buffers, H2D -> kernels -> D2H) at the committee sizes of C2 / C3 / C4.  Prints one JSON line
per committee; run under rocprofv3 --kernel-trace --stats to split the time by kernel.
Usage (GPU box): python tools/latency_probe.py [--samples 200] > gpurun_out/latency.jsonl"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=200)
    ap.add_argument("--only", default="100,1000,10000")
    args = ap.parse_args()
    from narwhal_amd import _lib, workload
    for nval in [int(x) for x in args.only.split(",")]:
        votes = 2 * nval // 3 + 1
        eng = _lib.Engine(device=0, key_window=-1)
        com = workload.make_committee(nval, eng)
        slots = eng.committee_load_np(com.pks, com.stake)
        ncerts = 16
        cs = workload.make_certificates(com, ncerts, votes, eng)
        zseed = os.urandom(32)
        lat = []
        for i in range(args.samples + 10):
            c = i % ncerts
            f, n = int(cs.cert_first[c]), int(cs.cert_n[c])
            t0 = time.perf_counter()
            cok, _, _ = eng.verify_certs_np(np.array([0], np.uint32), np.array([n], np.uint32), cs.sigs[f:f + n],
                                            slots[cs.signer[f:f + n]], cs.msgs[c:c + 1], zseed, c)
            dt = time.perf_counter() - t0
            assert cok[0] == 1
            if i >= 10:
                lat.append(dt)
        lat.sort()
        print(json.dumps({"validators": nval, "votes": votes, "key_window": eng.key_window(),
                          "p50_ms": lat[len(lat) // 2] * 1e3, "p99_ms": lat[int(len(lat) * 0.99)] * 1e3,
                          "min_ms": lat[0] * 1e3, "samples": len(lat)}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
