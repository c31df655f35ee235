"""Check the device math (compiled for the host by tools/hostcheck.hip) against the Python oracle.

Usage: python tools/hostcheck.py [n_random]
Test-only developer tool; the GPU parity tests live in tests/.
"""
import ctypes
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import ed25519_oracle as o  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libhostcheck.so"))
P, L = o.P, o.L


def b32(x):
    return (x % (1 << 256)).to_bytes(32, "little")


def call_fe(fn, *args):
    out = ctypes.create_string_buffer(32)
    fn(*[b32(a) for a in args], out)
    return int.from_bytes(out.raw, "little")


def check_field(rng, n):
    for _ in range(n):
        a, b, c = (rng.randrange(1 << 255) for _ in range(3))
        if rng.random() < 0.2:
            a = (1 << 255) - 1 - rng.randrange(40)   # non-canonical representatives
        assert call_fe(lib.hc_fe_mul, a, b) == a * b % P, "mul"
        assert call_fe(lib.hc_fe_sq, a) == a * a % P, "sq"
        assert call_fe(lib.hc_fe_mul_loose, a, b, c) == (a + b + c) * (a + b) % P, "mul loose"
        s, d = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        lib.hc_fe_add_sub(b32(a), b32(b), s, d)
        assert int.from_bytes(s.raw, "little") == (a + b) % P
        assert int.from_bytes(d.raw, "little") == (a - b) % P
    for _ in range(max(1, n // 20)):
        a = rng.randrange(1, P)
        assert call_fe(lib.hc_fe_invert, a) == pow(a, P - 2, P), "invert"
        assert call_fe(lib.hc_fe_invert_sg, a) == pow(a, P - 2, P), "invert (safegcd)"
    for a in [0, 1, 2, P - 1, P, P + 1, (1 << 255) - 1, 19, (1 << 254), (1 << 255) - 20]:
        assert call_fe(lib.hc_fe_invert_sg, a) == pow(a, P - 2, P), ("invert (safegcd)", a)
        assert call_fe(lib.hc_fe_pow22523, a) == pow(a, (P - 5) // 8, P), "pow22523"
    # all-ones limbs stress
    mx = (1 << 255) - 1
    assert call_fe(lib.hc_fe_mul_loose, mx, mx, mx) == (3 * mx) * (2 * mx) % P
    print("field ok")


def check_scalar(rng, n):
    for _ in range(n):
        x = rng.randrange(1 << 512)
        out = ctypes.create_string_buffer(32)
        lib.hc_sc_reduce512(x.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw, "little") == x % L
        a, b, c = (rng.randrange(1 << 256) for _ in range(3))
        lib.hc_sc_muladd(b32(a), b32(b), b32(c), out)
        assert int.from_bytes(out.raw, "little") == (a * b + c) % L
    for s in [0, L - 1, L, L + 1, 2**252, 2**253 - 1, 2**253, 2**256 - 1]:
        assert lib.hc_sc_is_canonical(b32(s)) == (1 if s < L else 0), s
    for x in [0, L - 1, L, 2 * L, (1 << 512) - 1]:
        out = ctypes.create_string_buffer(32)
        lib.hc_sc_reduce512(x.to_bytes(64, "little"), out)
        assert int.from_bytes(out.raw, "little") == x % L
    print("scalar ok")


def check_sha(rng, n):
    for _ in range(n):
        m = bytes(rng.randrange(256) for _ in range(96))
        out = ctypes.create_string_buffer(64)
        lib.hc_sha512_oneblock96(m, out)
        assert out.raw == o.sha512(m)
    for ln in [0, 1, 8, 32, 47, 48, 63, 64, 100, 111, 112, 127, 128, 200, 1000]:
        R = bytes(rng.randrange(256) for _ in range(32))
        A = bytes(rng.randrange(256) for _ in range(32))
        msg = bytes(rng.randrange(256) for _ in range(ln))
        out = ctypes.create_string_buffer(64)
        lib.hc_hram_generic(R, A, msg, ctypes.c_uint64(ln), out)
        assert out.raw == o.sha512(R + A + msg), ln
    print("sha ok")


def check_points(rng, n):
    for _ in range(n):
        ka, kb = rng.randrange(1, L), rng.randrange(1, L)
        A = o.pt_mul(ka, o.B_POINT)
        Bp = o.pt_mul(kb, o.B_POINT)
        if rng.random() < 0.3:
            A = o.pt_add(A, rng.choice(o.small_order_points()))
        ea, eb = o.pt_compress(A), o.pt_compress(Bp)
        k = rng.randrange(1 << 256)
        outs = [ctypes.create_string_buffer(32) for _ in range(4)]
        lib.hc_point_ops(ea, eb, b32(k), *outs)
        assert outs[0].raw == o.pt_compress(o.pt_add(A, Bp)), "add"
        assert outs[1].raw == o.pt_compress(o.pt_double(A)), "dbl"
        assert outs[2].raw == o.pt_compress(o.pt_add(A, Bp)), "madd"
        assert outs[3].raw == o.pt_compress(o.pt_mul(k, A)), "kmul"
        fused = ctypes.create_string_buffer(32)
        assert lib.hc_madd_fused(ea, eb, fused) == 1, "fused product groups"
        assert fused.raw == o.pt_compress(o.pt_add(A, Bp)), "madd (fused-carry products)"
    # decompression incl. non-canonical / invalid encodings
    cases = [bytes(32), b32(1), b32(P), b32(P + 1), b32(P + 18), b32((1 << 255) - 1),
             b32(1 | (1 << 255)), b32(P | (1 << 255))]
    for _ in range(n):
        cases.append(b32(rng.randrange(1 << 256)))
    for e in cases:
        out = ctypes.create_string_buffer(32)
        ok = lib.hc_decompress(e, out)
        ref = o.decompress(e)
        assert bool(ok) == (ref is not None), e.hex()
        if ref is not None:
            assert out.raw == o.pt_compress(ref), e.hex()
    print("points ok")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = random.Random(1)
    check_field(rng, n)
    check_scalar(rng, n)
    check_sha(rng, n // 4)
    check_points(rng, max(5, n // 20))
    print("ALL OK")


if __name__ == "__main__":
    main()
