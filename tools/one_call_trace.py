"""One-call latency anatomy (the shim's per-message paths): run under
``rocprofv3 --kernel-trace --memory-copy-trace`` and split each call into its GPU commands and the
gaps between them.  Calls: nw_verify_strict (cached key), nw_verify_batch of one 67-vote
certificate (cached keys), nw_verify_certs of the same certificate.  Each group of calls is
separated by a 20 ms host sleep so the trace can be cut into calls.
Usage (GPU box): rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o t --
    python3 tools/one_call_trace.py; then python3 tools/one_call_trace.py --analyze DIR"""
import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(reps):
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    from narwhal_amd import _lib, workload
    eng = _lib.Engine(device=0, key_window=-1)
    com = workload.make_committee(100, eng)
    slots = eng.committee_load_np(com.pks, com.stake)
    cs = workload.make_certificates(com, 4, 67, eng)
    msg, pk, sig = bytes(cs.msgs[0]), bytes(com.pks[cs.signer[0]]), bytes(cs.sigs[0])
    call = eng.prepare_batch_call([msg] * 67, [bytes(com.pks[k]) for k in cs.signer[:67]],
                                  [bytes(s) for s in cs.sigs[:67]])
    zseed = os.urandom(32)
    legs = {"strict": lambda: eng.verify_strict(msg, pk, sig),
            "batch67": lambda: call(zseed, 0),
            "certs67": lambda: eng.verify_certs_np(np.array([0], np.uint32), np.array([67], np.uint32),
                                                   cs.sigs[:67], slots[cs.signer[:67]], cs.msgs[:1], zseed, 0)}
    for name, fn in legs.items():
        for _ in range(3):
            fn()
        time.sleep(0.02)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            time.sleep(0.02)
        ts.sort()
        print(json.dumps({"leg": name, "p50_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3}), flush=True)


def analyze(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy")))
    rows.sort()
    calls, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > 5_000_000:   # > 5 ms idle: a new call
            calls.append(cur)
            cur = []
        cur.append(r)
    if cur:
        calls.append(cur)
    for c in calls[-60:]:
        t0 = c[0][0]
        parts = ["%s %.1f+%.1f" % (n, (s - t0) / 1e3, (e - s) / 1e3) for s, e, n in c]
        print("%.1f us | %s" % ((c[-1][1] - t0) / 1e3, " | ".join(parts)))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default=None)
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.reps)
