"""bench.py's worker_digest leg alone (GPU box), for A/B runs of the asynchronous digest path:
python tools/worker_leg.py [--prewarm N] > gpurun_out/worker_leg.json  (NWCRYPTO_LIB selects a variant
build).  --prewarm N first holds N asynchronous digest jobs at once, so the context's workspace pool
(one HIP stream each) has N members before the leg runs, as it has in bench.py after the host_fed and
msm legs (the worker-window bimodality)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prewarm", type=int, default=0)
    args = ap.parse_args()
    import bench
    from narwhal_amd import _lib
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0)
    if args.prewarm:
        jobs = [eng.sha512_many_submit([bytes(64 * (k + 1))]) for k in range(args.prewarm)]
        for j in jobs:
            j.wait()
    out = bench.worker_digest_leg(eng)
    out["prewarm"] = args.prewarm
    print(json.dumps({k: v for k, v in out.items() if k != "note"}))


if __name__ == "__main__":
    main()
