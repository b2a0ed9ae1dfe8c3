"""Generate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE ONLY).

    python -m oracle.gen_golden

ed25519 tuples (tests/golden/ed25519_vectors.json): every class of SURVEY.md §8c
"golden vectors to generate", each labelled.  Expected bits come from the
big-integer restatement of Go 1.18 crypto/ed25519.Verify (oracle/ed25519_go.py)
and are cross-checked against the C restatement (oracle/ed25519_port.c).
Classes (i)-(ix) — edge-case semantics are *derived from the Go 1.18 rule,
not reference-pinned* (the reference ships no ed25519 edge vectors).

Sign-bytes fixtures (tests/golden/signbytes_vectors.json): the five byte
vectors of types/vote_test.go:60-137 (data restated from the reference test)
plus commit-vote sign-bytes produced by oracle/signbytes.py.
"""
from __future__ import annotations

import hashlib
import json
import os
import random

from . import ed25519_go as E
from . import port
from .signbytes import PRECOMMIT_TYPE, ZERO_TIME, vote_sign_bytes

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")


def seed_of(tag: str, i: int) -> bytes:
    return hashlib.sha256(("%s-%d" % (tag, i)).encode()).digest()


def vote_msg(i: int, chain_id="test_chain_id", nil=False) -> bytes:
    h = 1 + i // 175
    bid = None if nil else (hashlib.sha256(h.to_bytes(8, "little")).digest(), 123,
                            hashlib.sha256(b"psh" + h.to_bytes(8, "little")).digest())
    ts = (1672531200 + i // 1000, (i % 1000) * 1_000_000)
    return vote_sign_bytes(chain_id, PRECOMMIT_TYPE, h, 0, bid, ts)


def enc_int(y: int, sign: int = 0) -> bytes:
    b = bytearray(y.to_bytes(32, "little"))
    b[31] |= sign << 7
    return bytes(b)


def sign_with_scalar(a: int, pub: bytes, msg: bytes, r: int) -> bytes:
    rb = E.encode(E.pt_mul(r, E.BASE))
    k = E.hram(rb, pub, msg)
    return rb + ((r + k * a) % E.L).to_bytes(32, "little")


def forge_for_torsion(pub: bytes, a: int, T, tor_order: int, msg: bytes, rng: random.Random):
    """Valid (Go-rule) signature for A = [a]B + T (T of small order): loop on the guess k mod ord(T)."""
    for _ in range(200):
        r = rng.randrange(1, E.L)
        j = rng.randrange(tor_order)
        Rpt = E.pt_add(E.pt_mul(r, E.BASE), E.pt_neg(E.pt_mul(j, T)))
        rb = E.encode(Rpt)
        k = E.hram(rb, pub, msg)
        if k % tor_order == j % tor_order:
            s = (r + k * a) % E.L
            sig = rb + s.to_bytes(32, "little")
            return sig
    raise RuntimeError("forge failed")


def main(n_valid=600, seed=0x5EED):
    rng = random.Random(seed)
    vecs = []

    def add(cls, pub, msg, sig):
        vecs.append({"class": cls, "pub": pub.hex(), "msg": msg.hex(), "sig": sig.hex(),
                     "valid": E.verify(pub, msg, sig) if len(sig) == 64 else False})

    keys = []
    for i in range(64):
        s = seed_of("golden-key", i)
        keys.append((s, E.pubkey_from_seed(s)))

    # (i) valid RFC 8032 signatures over CanonicalVote sign-bytes (+ nil votes (ix))
    for i in range(n_valid):
        s, pk = keys[i % len(keys)]
        m = vote_msg(i, nil=(i % 10 == 9))
        add("valid_vote" if i % 10 != 9 else "valid_nil_vote", pk, m, E.sign(s, m))
    # other message lengths (0..300 bytes, 1-3 SHA-512 blocks)
    for ln in [0, 1, 31, 32, 47, 48, 63, 64, 65, 111, 112, 113, 127, 128, 129, 175, 176, 239, 240, 241, 255, 256, 300]:
        s, pk = keys[ln % len(keys)]
        m = bytes(rng.randrange(256) for _ in range(ln))
        add("valid_len_%d" % ln, pk, m, E.sign(s, m))
    # RFC 8032 test 1/2
    sk1 = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    add("rfc8032_1", E.pubkey_from_seed(sk1), b"", E.sign(sk1, b""))
    sk2 = bytes.fromhex("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb")
    add("rfc8032_2", E.pubkey_from_seed(sk2), b"\x72", E.sign(sk2, b"\x72"))

    # (ii) bit flips in R, S, M, A
    for i in range(240):
        s, pk = keys[i % len(keys)]
        m = vote_msg(10_000 + i)
        sig = bytearray(E.sign(s, m))
        which = i % 4
        if which == 0:
            sig[rng.randrange(32)] ^= 1 << rng.randrange(8)
            add("flip_R", pk, m, bytes(sig))
        elif which == 1:
            sig[32 + rng.randrange(32)] ^= 1 << rng.randrange(8)
            add("flip_S", pk, m, bytes(sig))
        elif which == 2:
            mm = bytearray(m)
            mm[rng.randrange(len(mm))] ^= 1 << rng.randrange(8)
            add("flip_M", pk, bytes(mm), bytes(sig))
        else:
            pp = bytearray(pk)
            pp[rng.randrange(32)] ^= 1 << rng.randrange(8)
            add("flip_A", bytes(pp), m, bytes(sig))

    # (iii) S + L, S = L, S = L - 1, S with top bits set
    for i in range(24):
        s, pk = keys[i % len(keys)]
        m = vote_msg(20_000 + i)
        sig = E.sign(s, m)
        S = int.from_bytes(sig[32:], "little")
        add("S_plus_L", pk, m, sig[:32] + (S + E.L).to_bytes(32, "little"))
        add("S_eq_L", pk, m, sig[:32] + E.L.to_bytes(32, "little"))
        add("S_top_bits", pk, m, sig[:32] + (S | (1 << 253 + i % 3)).to_bytes(32, "little"))
    add("S_L_minus_1", keys[0][1], b"x", bytes(32) + (E.L - 1).to_bytes(32, "little"))
    add("S_zero", keys[0][1], b"x", bytes(32) + bytes(32))

    # (iv) non-canonical / off-curve R
    for i in range(24):
        s, pk = keys[i % len(keys)]
        m = vote_msg(30_000 + i)
        sig = E.sign(s, m)
        R = sig[:32]
        y = int.from_bytes(R, "little") & ((1 << 255) - 1)
        sgn = R[31] >> 7
        if y + E.P < (1 << 255):   # y >= p alias of the same y (only for y < 19)
            add("R_noncanon_y", pk, m, enc_int(y + E.P, sgn) + sig[32:])
        add("R_sign_flip", pk, m, bytes(R[:31]) + bytes([R[31] ^ 0x80]) + sig[32:])
        # off-curve R: a y that fails to decode
        yy = rng.randrange(E.P)
        while E.decode(enc_int(yy)) is not None:
            yy = rng.randrange(E.P)
        add("R_offcurve", pk, m, enc_int(yy) + sig[32:])
    # R encodings of small-order / identity points with y >= p and x=0 sign=1
    for y in range(0, 19):
        for sg in (0, 1):
            add("R_small_y_%d_%d" % (y, sg), keys[1][1], b"msg", enc_int(y + E.P, sg) + bytes(32))
            add("R_small_y_canon_%d_%d" % (y, sg), keys[1][1], b"msg", enc_int(y, sg) + bytes(32))

    # (v) small-order A (canonical and non-canonical encodings), valid-by-rule sigs
    small = E.small_order_points()
    for idx, T in enumerate(small):
        order = next(o for o in (1, 2, 4, 8) if E.pt_equal(E.pt_mul(o, T), E.IDENTITY))
        encs = [E.encode(T)]
        y = int.from_bytes(encs[0], "little") & ((1 << 255) - 1)
        if y + E.P < (1 << 255):
            encs.append(enc_int(y + E.P, encs[0][31] >> 7))
        x, yv, z, _ = T
        if x % E.P == 0:
            encs.append(enc_int(y, 1))       # x = 0 with the sign bit set (accepted by Go)
            if y + E.P < (1 << 255):
                encs.append(enc_int(y + E.P, 1))
        for j, pub in enumerate(encs):
            for t in range(3):
                m = b"small-order A %d/%d/%d" % (idx, j, t)
                sig = forge_for_torsion(pub, 0, T, order, m, rng)
                add("A_small_order", pub, m, sig)
                # and a random (almost surely invalid) one
                add("A_small_order_rand", pub, m, bytes(rng.randrange(256) for _ in range(32)) + sig[32:])

    # (vi) A with y >= p whose reduced y is on the curve, and non-square A
    for y in range(0, 19):
        for sg in (0, 1):
            pub = enc_int(y + E.P, sg)
            m = b"noncanon A %d %d" % (y, sg)
            sig = bytes(rng.randrange(256) for _ in range(32)) + (rng.randrange(E.L)).to_bytes(32, "little")
            add("A_noncanon_y", pub, m, sig)
    for i in range(16):
        yy = rng.randrange(E.P)
        while E.decode(enc_int(yy)) is not None:
            yy = rng.randrange(E.P)
        s, pk = keys[i]
        m = vote_msg(40_000 + i)
        add("A_offcurve", enc_int(yy, i & 1), m, E.sign(s, m))

    # (vii) mixed-order R (reject) and mixed-order A with consistent R (accept)
    T8 = next(T for T in small if not E.pt_equal(E.pt_mul(4, T), E.IDENTITY))
    for i in range(16):
        s, pk = keys[i]
        m = vote_msg(50_000 + i)
        sig = E.sign(s, m)
        R = E.decode(sig[:32])
        Rm = E.pt_add(R, E.pt_mul(1 + i % 7, T8))
        add("R_mixed_order", pk, m, E.encode(Rm) + sig[32:])
        a = rng.randrange(1, E.L)
        Tm = E.pt_mul(1 + i % 7, T8)
        order = next(o for o in (1, 2, 4, 8) if E.pt_equal(E.pt_mul(o, Tm), E.IDENTITY))
        Am = E.pt_add(E.pt_mul(a, E.BASE), Tm)
        pub = E.encode(Am)
        msg = b"mixed-order A %d" % i
        add("A_mixed_order", pub, msg, forge_for_torsion(pub, a, Tm, order, msg, rng))
        # a plain (cofactorless) signature with the prime-order part: rejected
        add("A_mixed_order_plain", pub, msg, sign_with_scalar(a, pub, msg, rng.randrange(1, E.L)))

    # (viii) short / long signatures (rejected by length, ed25519.go:150-152)
    for ln in (0, 1, 32, 63, 65):
        s, pk = keys[ln % 64]
        m = vote_msg(60_000 + ln)
        sig = E.sign(s, m)
        sig = (sig + b"\x00")[:ln] if ln <= 64 else sig + b"\x00"
        add("siglen_%d" % ln, pk, m, sig)

    # garbage
    for i in range(40):
        add("random", bytes(rng.randrange(256) for _ in range(32)), bytes(rng.randrange(256) for _ in range(rng.randrange(200))),
            bytes(rng.randrange(256) for _ in range(64)))

    # cross-check every 64-byte-sig vector against the C restatement
    for v in vecs:
        sig = bytes.fromhex(v["sig"])
        if len(sig) == 64:
            c = port.verify(bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), sig)
            assert c == v["valid"], ("oracle disagreement", v)

    os.makedirs(GOLDEN, exist_ok=True)
    with open(os.path.join(GOLDEN, "ed25519_vectors.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py", "semantics": "Go 1.18 crypto/ed25519.Verify (cofactorless; "
                   "S<L strict; permissive A decode; byte-compared R)", "pinning": "derived from the Go rule; "
                   "not reference-pinned for edge classes", "vectors": vecs}, f, indent=0)
    counts = {}
    for v in vecs:
        k = v["class"].split("_len_")[0]
        counts.setdefault(k, [0, 0])
        counts[k][0] += 1
        counts[k][1] += v["valid"]
    print(len(vecs), "vectors")
    for k in sorted(counts):
        print("  %-28s n=%4d valid=%4d" % (k, counts[k][0], counts[k][1]))

    # sign-bytes fixtures
    sb = {"generator": "oracle/gen_golden.py",
          "reference_vectors": [  # types/vote_test.go:60-137 (want bytes restated as data)
              {"chain_id": "", "type": 0, "height": 0, "round": 0,
               "want": "0d2a0b088092b8c398feffffff01"},
              {"chain_id": "", "type": 2, "height": 1, "round": 1,
               "want": "2108021101000000000000001901000000000000002a0b088092b8c398feffffff01"},
              {"chain_id": "", "type": 1, "height": 1, "round": 1,
               "want": "2108011101000000000000001901000000000000002a0b088092b8c398feffffff01"},
              {"chain_id": "", "type": 0, "height": 1, "round": 1,
               "want": "1f1101000000000000001901000000000000002a0b088092b8c398feffffff01"},
              {"chain_id": "test_chain_id", "type": 0, "height": 1, "round": 1,
               "want": "2e1101000000000000001901000000000000002a0b088092b8c398feffffff01320d746573745f636861696e5f6964"},
          ],
          "commit_votes": []}
    for i, (h, r, nil, cid, ts) in enumerate([(3, 0, False, "test_chain_id", (1672531200, 0)),
                                              (3, 0, True, "test_chain_id", (1672531200, 5)),
                                              (1, 1, False, "Lalande21185", (1672531200, 999999999)),
                                              (10**12, 7, False, "x" * 50, (2**40, 1)),
                                              (5, 0, False, "", ZERO_TIME)]):
        bid = None if nil else (hashlib.sha256(b"b%d" % i).digest(), 123, hashlib.sha256(b"p%d" % i).digest())
        sb["commit_votes"].append({"chain_id": cid, "height": h, "round": r, "nil": nil, "ts": list(ts),
                                   "hash": bid[0].hex() if bid else "", "psh_total": 123 if bid else 0,
                                   "psh_hash": bid[2].hex() if bid else "",
                                   "want": vote_sign_bytes(cid, PRECOMMIT_TYPE, h, r, bid, ts).hex()})
    with open(os.path.join(GOLDEN, "signbytes_vectors.json"), "w") as f:
        json.dump(sb, f, indent=1)


if __name__ == "__main__":
    main()
