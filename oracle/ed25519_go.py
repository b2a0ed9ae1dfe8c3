"""Big-integer restatement of Go 1.18 ``crypto/ed25519`` (TEST INFRASTRUCTURE ONLY).

Reference chain: ``crypto/ed25519/ed25519.go:148-155`` (``PubKey.VerifySignature``:
``len(sig) != 64`` -> false, then ``ed25519.Verify``) -> ``golang.org/x/crypto``
v0.1.0 (``go.mod:44``, ``ed25519_go113.go`` forwards to the stdlib) -> Go 1.18
``crypto/ed25519.Verify`` with ``crypto/internal/edwards25519`` (third-party to
the reference tree, restated here from its published algorithm):

1. ``len(sig) != 64 || sig[63] & 0xE0 != 0`` -> reject.
2. ``A = Point.SetBytes(pub)``: y = LE(pub) with bit 255 cleared, values >= p
   accepted and reduced; x = SqrtRatio((y^2-1), (d*y^2+1)) (non-negative root);
   non-square -> reject; if bit 255 set, x = -x (so x = 0 with the sign bit set
   is accepted).
3. ``k = SHA-512(sig[0:32] || pub || msg) mod L`` (``Scalar.SetUniformBytes``).
4. ``S = Scalar.SetCanonicalBytes(sig[32:64])``: S >= L -> reject.
5. ``R' = [k](-A) + [S]B`` (``VarTimeDoubleScalarBaseMult``; exact group law,
   no cofactor).
6. accept iff ``R'.Bytes() == sig[0:32]`` (canonical encoding: y reduced, bit 255
   = parity of x), so a non-canonical or off-curve R is always rejected.

Pure-Python loops: intended for small cases (fixtures, unit tests).  The fast
C restatement of the same rule is ``oracle/ed25519_port.c``.
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# Base point: y = 4/5, x even ("positive").
_BY = (4 * pow(5, P - 2, P)) % P


def _inv(z: int) -> int:
    return pow(z, P - 2, P)


def _sqrt_ratio(u: int, v: int):
    """Go ``field.Element.SqrtRatio``: (non-negative r, was_square)."""
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    u_neg = (-u) % P
    correct = check == u % P
    flipped = check == u_neg
    flipped_i = check == u_neg * SQRT_M1 % P
    if flipped or flipped_i:
        r = r * SQRT_M1 % P
    if r & 1:  # Absolute(): choose the non-negative (even) root
        r = (-r) % P
    return r, (correct or flipped)


def _bx() -> int:
    u = (_BY * _BY - 1) % P
    v = (D * _BY * _BY + 1) % P
    x, ok = _sqrt_ratio(u, v)
    assert ok
    return x


_BX = _bx()

# Extended coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, xy = T/Z.
IDENTITY = (0, 1, 1, 0)
BASE = (_BX, _BY, 1, _BX * _BY % P)


def pt_add(p, q):
    """Complete unified addition (a = -1 twisted Edwards, HWCD'08 'add-2008-hwcd-3')."""
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = t1 * D2 % P * t2 % P
    d = 2 * z1 * z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def pt_neg(p):
    x, y, z, t = p
    return ((-x) % P, y, z, (-t) % P)


def pt_mul(s: int, p):
    q = IDENTITY
    for bit in bin(s)[2:] if s > 0 else "":
        q = pt_add(q, q)
        if bit == "1":
            q = pt_add(q, p)
    return q


def pt_equal(p, q) -> bool:
    x1, y1, z1, _ = p
    x2, y2, z2, _ = q
    return (x1 * z2 - x2 * z1) % P == 0 and (y1 * z2 - y2 * z1) % P == 0


def pt_is_on_curve(p) -> bool:
    x, y, z, t = p
    zi = _inv(z)
    x, y = x * zi % P, y * zi % P
    return (-x * x + y * y - 1 - D * x * x % P * y * y) % P == 0


def encode(p) -> bytes:
    """Go ``Point.Bytes``: canonical y, bit 255 = parity of canonical x."""
    x, y, z, _ = p
    zi = _inv(z)
    x, y = x * zi % P, y * zi % P
    out = bytearray(y.to_bytes(32, "little"))
    out[31] |= (x & 1) << 7
    return bytes(out)


def decode(b: bytes):
    """Go ``Point.SetBytes`` (permissive): returns a point or None."""
    if len(b) != 32:
        return None
    y = (int.from_bytes(b, "little") & ((1 << 255) - 1)) % P
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x, ok = _sqrt_ratio(u, v)
    if not ok:
        return None
    if b[31] >> 7:
        x = (-x) % P
    return (x, y, 1, x * y % P)


def sc_reduce64(h: bytes) -> int:
    """Go ``Scalar.SetUniformBytes``: 64-byte LE mod L."""
    return int.from_bytes(h, "little") % L


def sc_canonical(b: bytes):
    """Go ``Scalar.SetCanonicalBytes``: None if s >= L."""
    s = int.from_bytes(b, "little")
    return s if s < L else None


def hram(r_bytes: bytes, pub: bytes, msg: bytes) -> int:
    return sc_reduce64(hashlib.sha512(r_bytes + pub + msg).digest())


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    """``PubKey.VerifySignature`` (crypto/ed25519/ed25519.go:148-155) -> Go 1.18 Verify."""
    if len(sig) != 64:                      # ed25519.go:150-152
        return False
    if len(pub) != 32:                      # Go panics; unreachable (crypto/encoding/codec.go:45-48)
        raise ValueError("ed25519: bad public key length")
    if sig[63] & 0xE0:
        return False
    a = decode(pub)
    if a is None:
        return False
    k = hram(sig[:32], pub, msg)
    s = sc_canonical(sig[32:])
    if s is None:
        return False
    r = pt_add(pt_mul(k, pt_neg(a)), pt_mul(s, BASE))
    return encode(r) == sig[:32]


# ---------------------------------------------------------------------------
# RFC 8032 key generation / signing (crypto/ed25519/ed25519.go:57-60,107-116).

def _clamp(h32: bytes) -> int:
    a = bytearray(h32)
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little")


def pubkey_from_seed(seed: bytes) -> bytes:
    h = hashlib.sha512(seed).digest()
    return encode(pt_mul(_clamp(h[:32]) % L, BASE))


def sign(seed: bytes, msg: bytes) -> bytes:
    """Deterministic RFC 8032 signature, as Go ``ed25519.Sign(NewKeyFromSeed(seed), msg)``."""
    h = hashlib.sha512(seed).digest()
    a = _clamp(h[:32]) % L
    pub = encode(pt_mul(a, BASE))
    r = sc_reduce64(hashlib.sha512(h[32:] + msg).digest())
    rb = encode(pt_mul(r, BASE))
    k = hram(rb, pub, msg)
    s = (r + k * a) % L
    return rb + s.to_bytes(32, "little")


# ---------------------------------------------------------------------------
# Helpers for edge-case fixture construction (not part of the verify rule).

def small_order_points():
    """The 8 points of order dividing 8, as extended points."""
    pts = []
    # y = 1 (identity), y = -1 (order 2), x = 0
    pts.append((0, 1, 1, 0))
    pts.append((0, P - 1, 1, 0))
    # order 4: y = 0, x = +-sqrt(-1)
    pts.append((SQRT_M1, 0, 1, 0))
    pts.append(((-SQRT_M1) % P, 0, 1, 0))
    # order 8: find y with x^2 = (y^2-1)/(dy^2+1) whose point has order 8
    # Points of order 8 satisfy [2]Q has order 4 i.e. y([2]Q) = 0.
    # Solve via torsion: take a point of order 8 = [L]*(random point) scaled.
    seen = set()
    q = None
    yv = 2
    while len(pts) < 8:
        pt = decode(yv.to_bytes(32, "little"))
        yv += 1
        if pt is None:
            continue
        t = pt_mul(L, pt)  # kill the prime-order part -> torsion component
        if pt_equal(t, IDENTITY):
            continue
        for j in range(8):
            c = pt_mul(j, t)
            e = encode(c)
            if e not in seen and not any(pt_equal(c, x) for x in pts):
                pts.append(c)
            seen.add(e)
        q = t
    return pts[:8]
