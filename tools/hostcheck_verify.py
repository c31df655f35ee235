"""Host-side check of the verify lane math + exact batch decomposition against the oracle's
literal restatement of dalek's verify_strict / verify_batch (test-only developer tool)."""
import ctypes
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import ed25519_oracle as o  # noqa: E402
import vectors  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libhostcheck.so"))
lib.hc_comb_words.restype = ctypes.c_size_t
lib.hc_build_comb.restype = ctypes.c_uint32
lib.hc_verify_lane.restype = ctypes.c_uint32
lib.hc_comb_words.argtypes = [ctypes.c_int]
KEY_W = int(os.environ.get("KEY_W", "8"))
F_S_OK, F_A_OK, F_MATCH, F_STRICT, F_SLOW = 1, 2, 4, 8, 0x1000

_tabs = {}


def comb(key, w=None):
    w = w or KEY_W
    if (key, w) not in _tabs:
        tab = (ctypes.c_uint32 * lib.hc_comb_words(w))()
        info = lib.hc_build_comb(key, tab, w)
        _tabs[(key, w)] = (tab, info)
    return _tabs[(key, w)]


BTAB, _ = comb(o.pt_compress(o.B_POINT), 16)


def lane(sig, pk, msg, zseed, counter, bidx):
    tab, info = comb(pk)
    q = ctypes.create_string_buffer(32)
    rbad = ctypes.c_int(0)
    f = lib.hc_verify_lane(sig, pk, msg, ctypes.c_uint64(len(msg)), info, tab, KEY_W, BTAB, zseed, counter,
                           ctypes.c_uint64(bidx), q, ctypes.byref(rbad))
    return f, q.raw, rbad.value


def batch_verdict(items, zseed, bidx):
    """Emulate k_cert_finalize from per-lane outputs."""
    bad, slow, tsum = False, False, 0
    acc = o.IDENTITY
    for i, (pk, sig, msg) in enumerate(items):
        f, q, rbad = lane(sig, pk, msg, zseed, i, bidx)
        if (f & (F_S_OK | F_A_OK)) != (F_S_OK | F_A_OK) or rbad:
            bad = True
        tsum += (f >> 8) & 7
        if f & F_SLOW and not rbad:
            slow = True
            acc = o.pt_add(acc, o.decompress(q))
    if bad:
        return False
    acc = o.pt_add(acc, o.pt_mul(tsum % 8, o.small_order_generator()))
    return o.pt_is_identity(acc)


def main():
    rng = random.Random(7)
    zseed = bytes(range(32))
    cases = vectors.adversarial_cases(rng)
    nstrict = nbatch = 0
    for name, pk, sig, msg in cases:
        f, _, _ = lane(sig, pk, msg, None, 0, 0)
        want = o.verify_strict(pk, msg, sig)
        assert bool(f & F_STRICT) == want, (name, hex(f), want)
        nstrict += 1
    # batches: mix honest signatures with each adversarial case
    honest = vectors.honest_cases(rng, 6)
    for idx, (name, pk, sig, msg) in enumerate(cases):
        if o.decompress(pk) is None:
            continue   # crypto::verify_batch rejects before dalek::verify_batch; covered by the API tests
        items = [(h[1], h[2], h[3]) for h in honest[:3]] + [(pk, sig, msg)]
        for bidx in (idx, idx + 1000):
            zs = o.batch_coefficients(zseed, bidx, len(items))
            want = o.verify_batch_z([m for _, _, m in items], [s for _, s, _ in items], [k for k, _, _ in items], zs)
            got = batch_verdict(items, zseed, bidx)
            assert got == want, (name, bidx, got, want)
            nbatch += 1
    for bidx in (3, 77):
        items = vectors.cancelling_pair(zseed, bidx, rng)
        zs = o.batch_coefficients(zseed, bidx, len(items))
        want = o.verify_batch_z([m for _, _, m in items], [s for _, s, _ in items], [k for k, _, _ in items], zs)
        assert want, "cancelling pair must pass dalek's equation"
        assert batch_verdict(items, zseed, bidx) == want
        assert not batch_verdict(items, zseed, bidx + 1)
        nbatch += 2
    print("strict cases ok:", nstrict, " batch cases ok:", nbatch)
    # signing
    for i in range(5):
        seed = bytes(rng.randrange(256) for _ in range(32))
        msg = bytes(rng.randrange(256) for _ in range(32))
        pk = ctypes.create_string_buffer(32)
        sg = ctypes.create_string_buffer(64)
        lib.hc_sign32(seed, msg, BTAB, pk, sg)
        assert pk.raw == o.public_from_seed(seed)
        assert sg.raw == o.sign(seed, msg)
    print("sign ok")


if __name__ == "__main__":
    main()
