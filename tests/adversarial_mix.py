"""BASELINE config C5's adversarial mix: replace a fraction of a
synthetic certificate set's signatures with a uniform mix of the verdict classes.  Test
infrastructure: uses the oracle's point arithmetic to build the mixed-order R of class (iii)."""
import hashlib

import numpy as np

import ed25519_oracle as o
import vectors

L = o.L
CLASSES = ["ii", "iii", "v", "vi", "vii", "viii", "ix"]   # signature-level; key-level: add_torsion_members


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


def add_torsion_members(cs, com, members_small, members_mixed):
    """Key-level classes at committee scale: committee members whose cached keys carry a torsion
    component.  Every vote of a member in ``members_small`` is re-signed under a small-order key
    A = T (class i: R = rB, S = r, so the batch residual h T is pure torsion); every vote of a member
    in ``members_mixed`` under the mixed-order key A' = aB + jT8 with the member's own scalar
    (class iv: honest R, S' = r + H(R||A'||M) a).  The nonce r of each vote is recovered from its
    honest signature (r = S - H(R||A||M) a mod l), so no point arithmetic runs per vote.
    Returns (committee with the torsion keys appended, {signature index: class}); ``cs.signer``
    and ``cs.sigs`` are rewritten in place to point at the appended keys."""
    import copy
    t8 = o.small_order_generator()
    small = [p for p in o.small_order_points() if not o.pt_is_identity(p)]
    new_pks, new_seeds, kinds = [], [], {}
    sigs = cs.sigs.copy()
    signer = cs.signer.copy()
    cert_of = np.repeat(np.arange(cs.ncerts), cs.cert_n.astype(np.int64))
    base = com.size
    for j, (mem, cls) in enumerate([(m, "i") for m in members_small] + [(m, "iv") for m in members_mixed]):
        seed = bytes(com.seeds[mem])
        a, _ = secret_scalar(seed)
        pk = bytes(com.pks[mem])
        if cls == "i":
            A2 = o.pt_compress(small[j % len(small)])
        else:
            A2 = o.pt_compress(o.pt_add(o.pt_mul(a, o.B_POINT), o.pt_mul(1 + 2 * (j % 4), t8)))
        new_pks.append(np.frombuffer(A2, np.uint8))
        new_seeds.append(com.seeds[mem])
        slot = base + j
        for i in np.nonzero(cs.signer == mem)[0]:
            msg = bytes(cs.msgs[cert_of[i]])
            R, S = bytes(sigs[i][:32]), int.from_bytes(bytes(sigs[i][32:]), "little")
            k = int.from_bytes(hashlib.sha512(R + pk + msg).digest(), "little") % L
            r = (S - k * a) % L
            if cls == "i":
                s2 = r
            else:
                k2 = int.from_bytes(hashlib.sha512(R + A2 + msg).digest(), "little") % L
                s2 = (r + k2 * a) % L
            sigs[i] = np.frombuffer(R + s2.to_bytes(32, "little"), np.uint8)
            signer[i] = slot
            kinds[int(i)] = cls
    cs.sigs, cs.signer = sigs, signer
    com2 = copy.copy(com)
    com2.pks = np.concatenate([com.pks, np.stack(new_pks)])
    com2.seeds = np.concatenate([com.seeds, np.stack(new_seeds)])
    com2.stake = np.concatenate([com.stake, np.ones(len(new_pks), com.stake.dtype)])
    return com2, kinds
