"""ZIP-215 ed25519 verification, big-integer restatement (TEST INFRASTRUCTURE ONLY).

The rule of the engine's OPT-IN batch mode (tmed_verify_batch_zip215), not of the reference's
default path.  The reference names ZIP-215 as the rule Tendermint adopts going forward
(``spec/core/encoding.md:52-54``, https://zips.z.cash/zip-0215) but its code verifies with Go
1.18 ``crypto/ed25519.Verify`` (``crypto/ed25519/ed25519.go:148-155``) — cofactorless, which
``oracle/ed25519_go.py`` restates.  /root/reference holds no ZIP-215 implementation and no
ZIP-215 vectors: **parity of this rule is unpinned**; it is restated from the ZIP's published
text:

1. ``len(sig) == 64`` (Tendermint's own length check, ``ed25519.go:150``).
2. A = decode(pub), R = decode(sig[0:32]) — both with the permissive decoding (non-canonical
   y >= p accepted and reduced, x = 0 with the sign bit accepted); a point not on the curve rejects.
3. S = LE(sig[32:64]) must be < L.
4. k = SHA-512(sig[0:32] || pub || M) mod L, over the ORIGINAL encodings.
5. accept iff [8]([S]B - R - [k]A) is the identity (cofactored: small-order components ignored).

Batch form (what the GPU's MSM checks, tmed/zip215 docs): with random 128-bit z_i,
sum_i z_i [8](S_i B - R_i - k_i A_i) = O  <=>  [8]([sum z_i S_i] B - sum [z_i] R_i - sum [z_i k_i] A_i) = O;
a failing batch is bisected and, at the leaves, decided by this single-signature rule, so the
per-signature bits equal ``verify`` exactly.
"""
from __future__ import annotations

from .ed25519_go import BASE, IDENTITY, L, decode, hram, pt_add, pt_equal, pt_mul, pt_neg, sc_canonical


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    if len(sig) != 64 or len(pub) != 32:
        return False
    a = decode(pub)
    r = decode(sig[:32])
    if a is None or r is None:
        return False
    s = sc_canonical(sig[32:])
    if s is None:
        return False
    k = hram(sig[:32], pub, msg)
    d = pt_add(pt_add(pt_mul(s, BASE), pt_neg(r)), pt_neg(pt_mul(k, a)))
    return pt_equal(pt_mul(8, d), IDENTITY)


def batch_equation(items, zs) -> bool:
    """sum z_i [8](S_i B - R_i - k_i A_i) == O over decodable items (pub, msg, sig) with S < L."""
    sb = 0
    acc = IDENTITY
    for (pub, msg, sig), z in zip(items, zs):
        a, r, s = decode(pub), decode(sig[:32]), sc_canonical(sig[32:])
        k = hram(sig[:32], pub, msg)
        sb = (sb + z * s) % L
        acc = pt_add(acc, pt_neg(pt_add(pt_mul(z, r), pt_mul(z * k % L, a))))
    acc = pt_add(acc, pt_mul(sb, BASE))
    return pt_equal(pt_mul(8, acc), IDENTITY)
