"""A/B of the uncached (MSM) verify path: msm leg wall time for the group count in NW_MSM_GROUPS."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from narwhal_amd import _lib
eng = _lib.Engine(device=0, key_window=-1)
for n, chunks in ((62500, 64), (62500, 8), (8192, 8)):
    r = bench.msm_leg(eng, n_sigs=n, chunks=chunks, reps=11)
    print(json.dumps({"lib": os.path.basename(os.environ.get("NWCRYPTO_LIB", "default")), "n_sigs": n, "chunks": chunks,
                      "msigs": r["value"] / 1e6, "ms": r["ms"]}), flush=True)
