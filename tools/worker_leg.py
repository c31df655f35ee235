"""bench.py's worker_digest leg alone (GPU box), for A/B runs of the asynchronous digest path:
python tools/worker_leg.py > gpurun_out/worker_leg.json  (NWCRYPTO_LIB selects a variant build)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (before libnwcrypto: shared HIP runtime)


def main():
    import bench
    from narwhal_amd import _lib
    torch.cuda.set_device(0)
    eng = _lib.Engine(device=0)
    out = bench.worker_digest_leg(eng)
    print(json.dumps({k: v for k, v in out.items() if k != "note"}))


if __name__ == "__main__":
    main()
