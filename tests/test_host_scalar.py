"""The scalar reduction k_verify runs (nw_scalar.h sc_reduce512: x mod l for the 512-bit
SHA-512(R || A || M), dalek's Scalar::from_hash), compiled for the host from the same
__host__ __device__ source and checked against Python integers: random 512-bit values, values next
to multiples of l and to the 2^252 folding boundary, and the extremes.  Host-only compile (~1 s);
the full device-math harness is tools/hostcheck.py.
"""
import ctypes
import os
import random
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = 2**252 + 27742317777372353535851937790883648493
HIPCC = "/opt/rocm/bin/hipcc"

SRC = r"""
#include <hip/hip_runtime.h>
#include <cstring>
#include "nw_scalar.h"
extern "C" void t_sc_reduce512(const unsigned char* in, unsigned char* out) {
    uint32_t x[16], r[8];
    std::memcpy(x, in, 64);
    nw::sc_reduce512(r, x);
    std::memcpy(out, r, 32);
}
extern "C" void t_sc_muladd(const unsigned char* a, const unsigned char* b, const unsigned char* c,
                            unsigned char* out) {
    uint32_t aw[8], bw[8], cw[8], r[8];
    std::memcpy(aw, a, 32); std::memcpy(bw, b, 32); std::memcpy(cw, c, 32);
    nw::sc_muladd(r, aw, bw, cw);
    std::memcpy(out, r, 32);
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    if not os.path.exists(HIPCC) or shutil.which("ld") is None:
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("sc")
    src = d / "sc.hip"
    src.write_text(SRC)
    so = d / "libsc.so"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", "--cuda-host-only",
                    "-I", os.path.join(ROOT, "narwhal_amd", "csrc"), str(src), "-o", str(so)],
                   check=True, capture_output=True)
    return ctypes.CDLL(str(so))


def _reduce(lib, x):
    out = ctypes.create_string_buffer(32)
    lib.t_sc_reduce512(x.to_bytes(64, "little"), out)
    return int.from_bytes(out.raw, "little")


def test_sc_reduce512_edges(lib):
    top = (2**512 - 1) // L * L
    for x in [0, 1, L - 1, L, L + 1, 2 * L - 1, 2 * L, 2**252 - 1, 2**252, 2**253, 2**256 - 1,
              2**504, 2**512 - 1, top, top - 1, top + L - 1 if top + L - 1 < 2**512 else top]:
        assert _reduce(lib, x) == x % L, hex(x)


def test_sc_reduce512_near_multiples_and_boundaries(lib):
    rng = random.Random(7)
    for _ in range(3000):
        m = rng.randrange(2**260)
        for d in (-2, -1, 0, 1, 2):
            x = m * L + d
            if 0 <= x < 2**512:
                assert _reduce(lib, x) == x % L
        for x in (2**252 + rng.randrange(2**126), 2**252 - rng.randrange(2**132), L + rng.randrange(2**20),
                  (rng.randrange(256) << 504) | rng.randrange(2**504), rng.randrange(2**253)):
            assert _reduce(lib, x) == x % L, hex(x)


def test_sc_reduce512_random(lib):
    rng = random.Random(8)
    for _ in range(20000):
        x = rng.randrange(2**512)
        assert _reduce(lib, x) == x % L


def test_sc_muladd_random(lib):
    rng = random.Random(9)
    out = ctypes.create_string_buffer(32)
    for _ in range(3000):
        a, b, c = (rng.randrange(2**256) for _ in range(3))
        lib.t_sc_muladd(*(v.to_bytes(32, "little") for v in (a, b, c)), out)
        assert int.from_bytes(out.raw, "little") == (a * b + c) % L
