#!/usr/bin/env python3
"""Golden tuples of the opt-in ZIP-215 mode (tests/golden/zip215_vectors.json) — TEST INFRASTRUCTURE.

Expected bits come from the big-integer restatement (oracle/zip215.py) and are cross-checked
against the C port (port_verify_zip215) and, for the Go column, oracle/ed25519_go.py.  The
reference holds no ZIP-215 vectors, so these are "derived from the ZIP-215 rule, parity
unpinned".  Every tuple of tests/golden/ed25519_vectors.json is included with its ZIP-215
answer (base_valid_zip215, aligned with that file), plus classes on which the two rules disagree:
  zip_R_mixed        R = rB + T (T of order 2/4/8) hashed into k, S = r + k a: Go rejects
                     (SB - kA = rB != R), ZIP-215 accepts ([8]T = O);
  zip_R_noncanon_id  R = identity encoded with y = 1 + p, A = aB + T_A, S = k a: Go rejects
                     (non-canonical bytes), ZIP-215 accepts (SB - kA - R = -kT_A);
  zip_R_negzero_id   the same with R = (x = 0, sign bit 1, y = 1);
  zip_small_both     A and R small-order, S = 0: ZIP-215 accepts ([8](-R - kA) = O);
and classes both rules reject (S + L, off-curve R, flipped bits)."""
from __future__ import annotations

import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ed25519_go as E  # noqa: E402
from oracle import port, zip215  # noqa: E402
from oracle.gen_golden import enc_int, seed_of  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(seed=0x215):
    rng = random.Random(seed)
    base = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_vectors.json")))["vectors"]
    vecs = []

    def add(cls, pub, msg, sig):
        z = zip215.verify(pub, msg, sig)
        assert z == port.verify_zip215(pub, msg, sig), cls
        vecs.append({"class": cls, "pub": pub.hex(), "msg": msg.hex(), "sig": sig.hex(),
                     "valid_zip215": int(z), "valid_go": int(E.verify(pub, msg, sig) if len(pub) == 32 else 0)})

    base_z = []
    for v in base:
        pub, msg, sig = bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])
        z = zip215.verify(pub, msg, sig)
        assert z == port.verify_zip215(pub, msg, sig), v["class"]
        base_z.append(int(z))
    small = E.small_order_points()
    tors = [T for T in small if not E.pt_equal(T, E.IDENTITY)]
    for i in range(24):
        a = rng.randrange(1, E.L)
        A = E.pt_mul(a, E.BASE)
        pub = E.encode(A)
        msg = b"zip215 R mixed %d" % i
        r = rng.randrange(1, E.L)
        Rm = E.pt_add(E.pt_mul(r, E.BASE), tors[i % len(tors)])
        rb = E.encode(Rm)
        k = E.hram(rb, pub, msg)
        add("zip_R_mixed", pub, msg, rb + ((r + k * a) % E.L).to_bytes(32, "little"))
    for i in range(12):
        a = rng.randrange(1, E.L)
        TA = tors[i % len(tors)]
        pub = E.encode(E.pt_add(E.pt_mul(a, E.BASE), TA))
        for cls, rb in (("zip_R_noncanon_id", enc_int(1 + E.P, 0)), ("zip_R_negzero_id", enc_int(1, 1))):
            msg = b"%s %d" % (cls.encode(), i)
            k = E.hram(rb, pub, msg)
            add(cls, pub, msg, rb + (k * a % E.L).to_bytes(32, "little"))
    for i, (TA, TR) in enumerate([(a, b) for a in small for b in small][:32]):
        pub, rb = E.encode(TA), E.encode(TR)
        add("zip_small_both", pub, b"small both %d" % i, rb + bytes(32))
    for i in range(12):
        s = seed_of("zipneg", i)
        pk = port.pubkey_from_seed(s)
        msg = b"zip neg %d" % i
        sig = port.sign(s, msg)
        add("zip_valid", pk, msg, sig)
        sl = int.from_bytes(sig[32:], "little") + E.L
        add("zip_S_plus_L", pk, msg, sig[:32] + sl.to_bytes(32, "little"))
        yy = rng.randrange(E.P)
        while E.decode(enc_int(yy)) is not None:
            yy = rng.randrange(E.P)
        add("zip_R_offcurve", pk, msg, enc_int(yy) + sig[32:])
        b = bytearray(sig)
        b[rng.randrange(64)] ^= 1 << rng.randrange(8)
        add("zip_flip", pk, msg, bytes(b))
    out = os.path.join(ROOT, "tests", "golden", "zip215_vectors.json")
    with open(out, "w") as f:
        json.dump({"generator": "oracle/gen_zip215.py", "semantics": "ZIP-215 (opt-in mode); valid_go = Go 1.18 rule",
                   "pinning": "derived from the ZIP-215 rule; parity unpinned (the reference holds no ZIP-215 "
                              "code or vectors; spec/core/encoding.md:52-54 only names it)",
                   "base_file": "tests/golden/ed25519_vectors.json",
                   "base_valid_zip215": base_z, "vectors": vecs}, f, indent=0)
    diff = sum(1 for v in vecs if v["valid_zip215"] != v["valid_go"])
    diff += sum(1 for v, z in zip(base, base_z) if v["valid"] != z)
    print("%d base + %d extra tuples, %d where ZIP-215 and Go disagree" % (len(base), len(vecs), diff))


if __name__ == "__main__":
    main()
