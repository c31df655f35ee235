"""One worker-digest window of C4's share (1,250 x 508,052-B batches) through nw_sha512_many_async,
timed piece by piece (GPU box): submit (packing into pinned memory + DMA enqueue), completion of the
job alone, and the same window through worker.DigestBatcher as bench.py's worker_digest leg pushes
it (max_bytes 256 / 1,024 MiB, depth 2 / 4).  Fresh host buffers each rep, as a worker receives them.  Prints JSON lines.
Usage: python tools/worker_window_probe.py [WINDOW] > gpurun_out/worker_window.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    from narwhal_amd import _lib, workload, worker
    win = int(sys.argv[1]) if len(sys.argv) > 1 else 1250
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0)
    host = workload.worker_batches_np(win)
    rows = [host[i] for i in range(win)]
    for _ in range(2):
        eng.sha512_many_submit(rows).wait()   # this size's workspace and pinned buffer
    for rep in range(4):
        msgs = [r.copy() for r in rows]
        t0 = time.perf_counter()
        job = eng.sha512_many_submit(msgs)
        t1 = time.perf_counter()
        job.wait()
        t2 = time.perf_counter()
        print(json.dumps({"what": "job", "window": win, "rep": rep, "submit_ms": (t1 - t0) * 1e3,
                          "job_ms": (t2 - t0) * 1e3, "MB": win * host.shape[1] / 1e6}), flush=True)
    for rep, (mb, depth) in enumerate([(256, 2), (1024, 2), (256, 4)] * 2):
        msgs = [r.copy() for r in rows]
        b = worker.DigestBatcher(eng, window=win, depth=depth, max_bytes=mb << 20)
        t0 = time.perf_counter()
        t_push = []
        for x in msgs:
            b.push(x)
            t_push.append(time.perf_counter())
        got = b.drain()
        t1 = time.perf_counter()
        assert len(got) == win
        print(json.dumps({"what": "batcher", "window": win, "rep": rep, "max_bytes_MiB": mb, "depth": depth,
                          "submissions": b.submissions, "push_loop_ms": (t_push[-1] - t0) * 1e3,
                          "total_ms": (t1 - t0) * 1e3, "batches_per_s": win / (t1 - t0)}), flush=True)


if __name__ == "__main__":
    main()
