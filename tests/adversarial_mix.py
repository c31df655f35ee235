"""BASELINE config C5's adversarial mix: replace a fraction of a
synthetic certificate set's signatures with a uniform mix of the verdict classes.  Test
infrastructure: uses the oracle's point arithmetic to build the mixed-order R of class (iii)."""
import hashlib

import numpy as np

import ed25519_oracle as o
import vectors

L = o.L
CLASSES = ["ii", "iii", "v", "vi", "vii", "viii", "ix"]


def secret_scalar(seed: bytes):
    h = hashlib.sha512(seed).digest()
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def make_adversarial(cs, com, frac: float, rng: np.random.Generator):
    """Replace ``frac`` of cs.sigs (in place) with (keys stay honest committee keys):
      ii    R = identity, S = k a              (strict reject: R small order; batch accept)
      iii   R' = r B + T8, S = r + k' a         (strict reject; batch accept iff 8 | z)
      v     S + l                               (reject: non-canonical S)
      vi    S with the top three bits set       (reject: ed25519 high-bit check)
      vii   R with one flipped bit              (undecodable or mismatching R: reject)
      viii  R = a non-canonical encoding        (decodes, never matches: reject)
      ix    signature of another message        (reject)
    Returns {signature index: class}."""
    n = cs.nsigs
    idx = rng.choice(n, size=max(1, int(n * frac)), replace=False)
    sigs = cs.sigs.copy()
    t8 = o.small_order_generator()
    nonc = vectors.noncanonical_encodings()
    cert_of = np.repeat(np.arange(cs.ncerts), cs.cert_n.astype(np.int64))
    kinds = {}
    for j, i in enumerate(idx):
        cls = CLASSES[j % len(CLASSES)]
        kinds[int(i)] = cls
        seed = bytes(com.seeds[cs.signer[i]])
        pk = bytes(com.pks[cs.signer[i]])
        msg = bytes(cs.msgs[cert_of[i]])
        s = bytearray(sigs[i])
        if cls == "ii":
            R = (1).to_bytes(32, "little")
            a, _ = secret_scalar(seed)
            k = int.from_bytes(hashlib.sha512(R + pk + msg).digest(), "little") % L
            s = bytearray(R + (k * a % L).to_bytes(32, "little"))
        elif cls == "iii":
            a, prefix = secret_scalar(seed)
            r = int.from_bytes(hashlib.sha512(prefix + msg).digest(), "little") % L
            Rp = o.pt_compress(o.pt_add(o.pt_mul(r, o.B_POINT), t8))
            k = int.from_bytes(hashlib.sha512(Rp + pk + msg).digest(), "little") % L
            s = bytearray(Rp + ((r + k * a) % L).to_bytes(32, "little"))
        elif cls == "v":
            sv = int.from_bytes(bytes(s[32:]), "little") + L
            s[32:] = sv.to_bytes(32, "little")
        elif cls == "vi":
            s[63] |= 0xE0
        elif cls == "vii":
            s[int(rng.integers(0, 31))] ^= 1 << int(rng.integers(0, 8))
        elif cls == "viii":
            s[:32] = nonc[j % len(nonc)]
        else:
            s = bytearray(o.sign(seed, msg[::-1]))
        sigs[i] = np.frombuffer(bytes(s), np.uint8)
    cs.sigs = sigs
    return kinds
