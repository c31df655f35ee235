"""Latency of strict verify with keys outside the committee cache (k_verify_var + k_finish), one
ABI call per sample, at call sizes around the quad / lane kernel switch (4,096 signatures).
Usage (GPU box): python tools/strict_latency.py [--samples 200] > gpurun_out/strict_latency.jsonl"""
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
    ap.add_argument("--sizes", default="1,16,17,64,256,1024,4096,4097")
    args = ap.parse_args()
    from narwhal_amd import _lib
    eng = _lib.Engine(device=0, key_window=-1)
    for n in [int(x) for x in args.sizes.split(",")]:
        seeds = np.frombuffer(os.urandom(32 * n), np.uint8).reshape(n, 32)
        msgs = np.frombuffer(os.urandom(32 * n), np.uint8).reshape(n, 32)
        pks, sigs = eng.sign_many_np(seeds, msgs)
        m, k, s = [bytes(x) for x in msgs], [bytes(x) for x in pks], [bytes(x) for x in sigs]
        assert eng.verify_strict_many(m, k, s) == [True] * n
        for _ in range(5):
            eng.verify_strict_many(m, k, s)
        ts = []
        for _ in range(args.samples):
            t0 = time.perf_counter()
            eng.verify_strict_many(m, k, s)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(json.dumps({"sigs": n, "p50_ms": ts[len(ts) // 2] * 1e3, "p99_ms": ts[int(len(ts) * 0.99)] * 1e3,
                          "min_ms": ts[0] * 1e3, "samples": args.samples}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
