"""Kernel-time probe of the uncached batch path with an experimental library (NWCRYPTO_LIB):
calls nw_verify_batches_pk on the msm leg's workload without checking verdicts (run under rocprofv3)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from narwhal_amd import _lib, workload
eng = _lib.Engine(device=0, key_window=-1)
n, chunks = 62500, 64
seeds = np.frombuffer(workload._chacha20_keystream(32 * n), np.uint8).reshape(n, 32)[::-1].copy()
msgs = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8).copy()
pks, sigs = eng.sign_many_np(seeds, msgs)
counts = [(n * (c + 1)) // chunks - (n * c) // chunks for c in range(chunks)]
call = eng.prepare_batches_pk_call(counts, msgs, pks, sigs)
for r in range(6):
    ok = call(bytes(32), r * chunks)
print("accepted batches:", int(ok.sum()), "of", chunks)
