"""Where the batched worker digest spends its time (GPU box): per window size, the host time of
nw_sha512_many_async (staging memcpy + enqueue), the time to completion of one job alone, and two
jobs in flight at once; batches reused vs freshly allocated.  Prints JSON lines.
Usage: python tools/worker_probe.py > gpurun_out/worker_probe.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    from narwhal_amd import _lib, workload
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0)
    host = workload.worker_batches_np(256)
    for win in (1, 32, 128, 256):
        rows = [host[i] for i in range(win)]
        for rep in range(2):
            eng.sha512_many_submit(rows).wait()   # warm this size's workspace
        for kind in ("reused", "fresh"):
            subs, alone = [], []
            for rep in range(5):
                msgs = rows if kind == "reused" else [r.copy() for r in rows]
                t0 = time.perf_counter()
                job = eng.sha512_many_submit(msgs)
                t1 = time.perf_counter()
                job.wait()
                t2 = time.perf_counter()
                subs.append((t1 - t0) * 1e3)
                alone.append((t2 - t0) * 1e3)
            t0 = time.perf_counter()
            j1 = eng.sha512_many_submit(rows if kind == "reused" else [r.copy() for r in rows])
            j2 = eng.sha512_many_submit(rows if kind == "reused" else [r.copy() for r in rows])
            j1.wait()
            t1 = time.perf_counter()
            j2.wait()
            t2 = time.perf_counter()
            print(json.dumps({"window": win, "buffers": kind, "submit_ms": sorted(subs)[2], "job_ms": sorted(alone)[2],
                              "two_jobs_first_ms": (t1 - t0) * 1e3, "two_jobs_both_ms": (t2 - t0) * 1e3,
                              "MB": win * host.shape[1] / 1e6}), flush=True)


if __name__ == "__main__":
    main()
