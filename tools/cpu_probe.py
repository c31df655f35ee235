"""Host-CPU probe for the CPU baseline (runs on the GPU box): affinity, cgroup CPU quota, and the
oracle's C restatement rate at several thread counts on C2-shaped certificates (no GPU use)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import ed25519_oracle as o  # noqa: E402
import nw_ref  # noqa: E402


def quota():
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(p).read().split()
            return None if q == "max" else float(q) / float(per)
        except Exception:
            pass
    return None


class Com:
    pass


class Cs:
    pass


def main():
    n_val, votes, ncerts = 100, 67, 4096
    seeds = [bytes([i % 256, i // 256]) * 16 for i in range(n_val)]
    com = Com()
    com.pks = np.frombuffer(b"".join(o.public_from_seed(s) for s in seeds), np.uint8).reshape(n_val, 32)
    cs = Cs()
    cs.cert_n = np.full(ncerts, votes, np.uint32)
    cs.cert_first = (np.arange(ncerts) * votes).astype(np.uint32)
    cs.msgs = np.frombuffer(os.urandom(32 * ncerts), np.uint8).reshape(ncerts, 32).copy()
    cs.signer = (np.arange(ncerts * votes) % n_val).astype(np.uint32)
    # one signature per (validator, certificate) would take minutes in Python; sign 64 distinct
    # messages and reuse them (the verify work per certificate is the same)
    uniq = 64
    sig_tab = {}
    for c in range(uniq):
        for v in range(n_val):
            sig_tab[(c, v)] = o.sign(seeds[v], bytes(cs.msgs[c]))
    for c in range(ncerts):
        cs.msgs[c] = cs.msgs[c % uniq]
    cs.sigs = np.frombuffer(b"".join(sig_tab[(c % uniq, int(cs.signer[c * votes + k]))]
                                     for c in range(ncerts) for k in range(votes)), np.uint8).reshape(-1, 64)
    out = {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(), "cgroup_quota_cpus": quota(),
           "rates": {}}
    for th in (1, 8, 16, 32, 64, 128, 256):
        if th > out["affinity"]:
            break
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < 2.0:
            sel = list(range(0, min(ncerts, max(64, 8 * th))))
            assert all(nw_ref.verify_certs(cs, com, sel, bytes(32), th))
            done += len(sel) * votes
        out["rates"][th] = done / (time.perf_counter() - t0)
        print(th, out["rates"][th], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
