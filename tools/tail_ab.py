"""Small-call latency A/B (run once per library, NWCRYPTO_LIB picks a variant): one 67-vote batch
through crypto::Signature::verify_batch's call (prepare_batch_call, keys cached), one certificate
through nw_verify_certs, one strict signature.  Prints one JSON line.
Usage (GPU box): NWCRYPTO_LIB=... python tools/tail_ab.py --tag NAME [--samples 400]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def p50(fn, n):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="default")
    ap.add_argument("--samples", type=int, default=400)
    args = ap.parse_args()
    from narwhal_amd import _lib, workload
    eng = _lib.Engine(device=0, key_window=-1)
    com = workload.make_committee(100, eng)
    slots = np.asarray(eng.committee_load_np(com.pks, com.stake), np.uint32)
    cs = workload.make_certificates(com, 4, 67, eng)
    zseed = os.urandom(32)
    n = int(cs.cert_n[0])
    out = {"tag": args.tag}
    msg, pk, sig = bytes(cs.msgs[0]), bytes(com.pks[cs.signer[0]]), bytes(cs.sigs[0])
    out["strict_cached"] = p50(lambda: eng.verify_strict(msg, pk, sig), args.samples)
    call = eng.prepare_batch_call([msg] * n, [bytes(com.pks[k]) for k in cs.signer[:n]], [bytes(x) for x in cs.sigs[:n]])
    assert call(zseed, 0)
    out["batch_cached_67"] = p50(lambda: call(zseed, 0), args.samples)
    first, cnt = np.array([0], np.uint32), np.array([n], np.uint32)
    sg, sl, ms = cs.sigs[:n].copy(), slots[cs.signer[:n]].copy(), cs.msgs[:1].copy()
    assert eng.verify_certs_np(first, cnt, sg, sl, ms, zseed, 0)[0][0] == 1
    out["cert_67"] = p50(lambda: eng.verify_certs_np(first, cnt, sg, sl, ms, zseed, 0), args.samples)
    bad = cs.sigs[:n].copy()
    bad[3, 40] ^= 1
    bad[9, 40] ^= 1
    assert eng.verify_certs_np(first, cnt, bad, sl, ms, zseed, 0)[0][0] == 0
    out["cert_67_two_bad"] = p50(lambda: eng.verify_certs_np(first, cnt, bad, sl, ms, zseed, 0), args.samples // 4)
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
