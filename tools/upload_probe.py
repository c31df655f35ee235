"""Host -> HBM upload of the C4 worker-batch share (1,250 x 508,052 B): where the time goes.

    python3 tools/upload_probe.py [--threads 8,16] [--chunk-mib 32]

Times, per configuration (median of 5): staging alone (pageable -> pinned, host threads), the DMA
alone (pinned -> HBM on a copy stream), and both pipelined chunk by chunk as bench.py's
BatchUploader does.  One JSON line per configuration."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--chunk-mib", default="8,32")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from narwhal_amd import workload
    host = workload.worker_batches_np(1250).reshape(-1)
    n = host.shape[0]
    pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
    pn = pinned.numpy()
    dbuf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    cs = torch.cuda.Stream()

    def med(f):
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e3

    def dma():
        with torch.cuda.stream(cs):
            dbuf.copy_(pinned, non_blocking=True)

    out = {"bytes": n, "dma_only_ms": med(dma), "pinned_is_pinned": bool(pinned[1000:].is_pinned())}
    print(json.dumps(out), flush=True)
    for th in [int(x) for x in args.threads.split(",")]:
        pool = ThreadPoolExecutor(th)
        for cm in [int(x) for x in args.chunk_mib.split(",")]:
            ch = cm << 20
            bounds = list(range(0, n, ch)) + [n]

            def stage_only():
                list(pool.map(lambda ab: np.copyto(pn[ab[0]:ab[1]], host[ab[0]:ab[1]]), zip(bounds, bounds[1:])))

            def both():
                futs = [pool.submit(np.copyto, pn[a:b], host[a:b]) for a, b in zip(bounds, bounds[1:])]
                with torch.cuda.stream(cs):
                    for f, a, b in zip(futs, bounds, bounds[1:]):
                        f.result()
                        dbuf[a:b].copy_(pinned[a:b], non_blocking=True)

            r = {"threads": th, "chunk_mib": cm, "stage_only_ms": med(stage_only), "pipelined_ms": med(both)}
            t0 = time.perf_counter()
            both()
            r["pipelined_host_return_ms"] = (time.perf_counter() - t0) * 1e3
            torch.cuda.synchronize()
            print(json.dumps(r), flush=True)
        pool.shutdown()
    assert bool((dbuf[-1000:].cpu().numpy() == host[-1000:]).all())


if __name__ == "__main__":
    main()
