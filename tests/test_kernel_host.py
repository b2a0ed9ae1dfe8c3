"""The exact kernel source (tendermint-fork_amd/csrc/*.h) compiled for the CPU
(tests/native/hostsim.cpp, test-only) against the oracle — catches arithmetic
bugs without a GPU.  The GPU parity proper is tests/test_gpu_verify.py."""
import ctypes
import hashlib
import random

import numpy as np
import pytest

from oracle import ed25519_go as E
from oracle import port

VP = ctypes.c_void_p


def _p(a):
    return a.ctypes.data_as(VP)


def _fe(l, op, a, b):
    o = ctypes.create_string_buffer(32)
    l.hostsim_fe_op(op, a.to_bytes(32, "little"), b.to_bytes(32, "little"), o)
    return int.from_bytes(o.raw, "little")


def test_field_ops_vs_bigint(hostsim):
    P = E.P
    rng = random.Random(11)
    edge = [0, 1, 2, 19, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**255 - 20, 2**254, 2**26 - 1, 2**51]
    vals = edge + [rng.randrange(2**255) for _ in range(120)]
    for a in vals:
        for b in edge[:6] + [rng.randrange(2**255)]:
            A, B = a % P, b % P
            exp = {0: A * B % P, 1: A * A % P, 2: pow(A, P - 2, P), 3: pow(A, (P - 5) // 8, P), 4: (A + B) % P,
                   5: (A - B) % P, 6: 2 * A * A % P, 7: (2 * A + B) ** 2 % P, 8: (2 * A + B) ** 2 % P,
                   9: pow(A, P - 2, P)}
            for op, e in exp.items():
                assert _fe(hostsim, op, a, b) == e, (op, hex(a), hex(b))


def test_binary_gcd_inversion(hostsim):
    """fe25519.h fe_invert_bgcd (the batched finish's inversion): equal to z^(p-2) on random values,
    powers of two and their neighbours, values near p and 0 (0 -> 0, as z^(p-2))."""
    P = E.P
    rng = random.Random(23)
    vals = [0, 1, 2, 3, P - 1, P - 2, P, P + 1, 2**255 - 1, 2**254, 2**64, 2**64 - 1, 2**30, 2**30 - 1, 2**60 + 1]
    vals += [2**rng.randrange(255) for _ in range(60)] + [(2**rng.randrange(255)) - 1 for _ in range(60)]
    vals += [rng.randrange(2**rng.randrange(1, 256)) for _ in range(400)] + [P - rng.randrange(2**40) for _ in range(40)]
    for a in vals:
        assert _fe(hostsim, 9, a, 0) == pow(a % P, P - 2, P), hex(a)


def test_pack256_roundtrip_at_the_limb_extremes(hostsim):
    """fe_pack256 / fe_unpack256 (the 128-B per-lane table entries of verify_main_hs_kernel):
    for 2-sums of carried values at the ends of their limb ranges, the unpacked value is congruent
    mod p, its limbs sit in [0, 2^26) / [0, 2^25) (limb 9 in [-2, 2^25]), and it multiplies
    correctly as a fe_mul operand."""
    P = E.P
    off = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    # carried ranges (fe_carry64): even [-2^25, 2^25), odd [-2^24, 2^24), limbs 1 and 5 one wider
    lo = [-(2**25) if i % 2 == 0 else -(2**24) for i in range(10)]
    hi = [2**25 - 1 if i % 2 == 0 else 2**24 - 1 for i in range(10)]
    lo[1] -= 1; lo[5] -= 1; hi[1] += 1; hi[5] += 1
    rng = random.Random(5)
    cases = [[2 * lo[i] for i in range(10)], [2 * hi[i] for i in range(10)], [0] * 10,
             [2 * lo[i] if i % 2 else 2 * hi[i] for i in range(10)], [2 * hi[i] if i % 2 else 2 * lo[i] for i in range(10)]]
    for i in range(10):
        for v in (2 * lo[i], 2 * hi[i]):
            c = [0] * 10
            c[i] = v
            cases.append(c)
    cases += [[rng.randint(2 * lo[i], 2 * hi[i]) for i in range(10)] for _ in range(800)]
    g = rng.randrange(P)
    out = (ctypes.c_int32 * 10)()
    prod = ctypes.create_string_buffer(32)
    for c in cases:
        hostsim.hostsim_pack256((ctypes.c_int32 * 10)(*c), g.to_bytes(32, "little"), out, prod)
        val = sum(x << o for x, o in zip(c, off))
        u = list(out)
        for i in range(9):
            assert 0 <= u[i] < (2**25 if i % 2 else 2**26), (c, u)
        assert -2 <= u[9] <= 2**25, (c, u)
        assert sum(x << o for x, o in zip(u, off)) % P == val % P
        assert int.from_bytes(prod.raw, "little") == val * g % P


def test_sha512_and_reduce(hostsim):
    rng = random.Random(5)
    for n in [0, 1, 17, 111, 112, 113, 127, 128, 129, 200, 239, 240, 241, 300, 400]:
        m = bytes(rng.randrange(256) for _ in range(n))
        o = ctypes.create_string_buffer(64)
        hostsim.hostsim_sha512(m, n, o)
        assert o.raw == hashlib.sha512(m).digest()
        r = ctypes.create_string_buffer(32)
        hostsim.hostsim_sc_reduce(o.raw, r)
        assert int.from_bytes(r.raw, "little") == int.from_bytes(o.raw, "little") % E.L
    for x in [b"\xff" * 64, bytes(64), E.L.to_bytes(64, "little"), (E.L - 1).to_bytes(64, "little"),
              (2 * E.L).to_bytes(64, "little"), (E.L * (2**259 - 1)).to_bytes(64, "little")]:
        r = ctypes.create_string_buffer(32)
        hostsim.hostsim_sc_reduce(x, r)
        assert int.from_bytes(r.raw, "little") == int.from_bytes(x, "little") % E.L


def test_decode_matches_go_rule(hostsim):
    rng = random.Random(9)
    cands = [bytes(32), bytes(31) + b"\x80"] + [rng.randbytes(32) for _ in range(80)]
    cands += [E.encode(q) for q in E.small_order_points()]
    cands += [(y + E.P).to_bytes(32, "little") for y in range(19)]
    for p in cands:
        o = ctypes.create_string_buffer(32)
        ok = hostsim.hostsim_decode(p, o)
        pt = E.decode(p)
        assert bool(ok) == (pt is not None), p.hex()
        if pt is not None:
            assert o.raw == E.encode(pt)


def _verify(l, pubs, sigs, msgs, offs, group=16):
    n = len(pubs)
    out = np.zeros(n, np.uint8)
    if group == "hs":  # main variant 6 (default): half-size scalars, verify_hs.h, radix-2^26 B windows
        l.hostsim_verify_batch_hs(_p(pubs), _p(sigs), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(out), None)
        return out
    if group == "hs16":  # the same with the radix-2^16 B windows (no 8.6-GB tables)
        l.hostsim_verify_batch_hs16(_p(pubs), _p(sigs), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(out), None)
        return out
    if group == "b16":  # main-kernel variant 5: radix-2^16 B windows from the 32769-entry table
        l.hostsim_verify_batch_b16(_p(pubs), _p(sigs), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(out))
        return out
    l.hostsim_verify_batch_g(_p(pubs), _p(sigs), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(out),
                             ctypes.c_int(group))
    return out


@pytest.mark.parametrize("group", [0, 1, 5, 16, "b16", "hs", "hs16"])
def test_golden_vectors_hostsim(hostsim, golden, group):
    """Every golden tuple, with per-signature encoding (group 0) and through the batched
    finish (Montgomery inversion over groups of 1, 5 and 16 signatures, partial last group);
    "b16": the radix-2^16 B-window variant of the main kernel."""
    vs = [v for v in golden if len(v["sig"]) == 128]
    pubs = np.array([np.frombuffer(bytes.fromhex(v["pub"]), np.uint8) for v in vs])
    sigs = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs])
    ms = [bytes.fromhex(v["msg"]) for v in vs]
    offs = np.zeros(len(vs) + 1, np.uint32)
    offs[1:] = np.cumsum([len(m) for m in ms])
    msgs = np.frombuffer(b"".join(ms) + b"\0", np.uint8)
    out = _verify(hostsim, pubs, sigs, msgs, offs, group)
    exp = np.array([v["valid"] for v in vs], np.uint8)
    bad = [vs[i]["class"] for i in np.nonzero(out != exp)[0]]
    assert not bad, bad


def test_sign_matches_oracle(hostsim):
    rng = np.random.default_rng(2)
    n = 96
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(0, 260, n)
    offs = np.zeros(n + 1, np.uint32)
    offs[1:] = np.cumsum(lens)
    msgs = rng.integers(0, 256, int(offs[-1]) + 1, dtype=np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    pub = np.zeros((n, 32), np.uint8)
    hostsim.hostsim_sign_batch(_p(seeds), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(sig), _p(pub))
    for i in range(n):
        m = msgs[offs[i]:offs[i + 1]].tobytes()
        assert sig[i].tobytes() == port.sign(seeds[i].tobytes(), m)
        assert pub[i].tobytes() == port.pubkey_from_seed(seeds[i].tobytes())


@pytest.mark.parametrize("fn", ["hostsim_verify_comb_batch", "hostsim_verify_comb_batch16", "hostsim_verify_comb_lat"])
def test_comb_path_hostsim(hostsim, golden, fn):
    """Key-cached (radix-256 comb) verification, host build of the kernel code, vs the oracle:
    golden tuples grouped by key (incl. small-order, non-canonical and undecodable keys).
    _lat: latency mode (8 partial comb sums + cross-lane tree, strict R decode + projective
    compare instead of the inversion) — covers the non-canonical / off-curve / x=0-sign R
    classes of the golden set."""
    per = {}
    for v in golden:  # up to 5 tuples of every edge class, so each R / A / S class is hit
        if len(v["sig"]) == 128 and len(per.setdefault(v["class"], [])) < 5:
            per[v["class"]].append(v)
    vs = [v for c in sorted(per) for v in per[c]]
    keys = sorted({v["pub"] for v in vs})
    kidx = {k: i for i, k in enumerate(keys)}
    karr = np.array([np.frombuffer(bytes.fromhex(k), np.uint8) for k in keys])
    idx = np.array([kidx[v["pub"]] for v in vs], np.uint32)
    sigs = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs])
    ms = [bytes.fromhex(v["msg"]) for v in vs]
    offs = np.zeros(len(vs) + 1, np.uint32)
    offs[1:] = np.cumsum([len(m) for m in ms])
    msgs = np.frombuffer(b"".join(ms) + b"\0", np.uint8)
    out = np.zeros(len(vs), np.uint8)
    getattr(hostsim, fn)(_p(karr), ctypes.c_size_t(len(keys)), _p(idx), _p(sigs), _p(msgs), _p(offs),
                         ctypes.c_size_t(len(vs)), _p(out))
    exp = np.array([v["valid"] for v in vs], np.uint8)
    assert (out == exp).all(), [vs[i]["class"] for i in np.nonzero(out != exp)[0]]
    assert exp.sum() > 10 and (exp == 0).sum() > 10


def test_halfsize_lattice(hostsim):
    """verify_hs.h sc_halfsize: c = d k (mod 8L), d odd, both within the window count's range
    (|x| < 2^(4W-1), the top digit taking the recoding's carry); W = 64 only for the (k, 1)
    fallback; typical W is 32..33."""
    L = E.L
    rng = random.Random(3)
    ks = [0, 1, 2, 3, 8, 16, L - 1, L - 2, 2**127, 2**128 - 1, 2**128, 2**200, 2**252 - 1, 5 * 2**128 + 3]
    ks += [rng.randrange(L) for _ in range(4000)]
    ws = []
    for k in ks:
        c, d = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        neg = ctypes.c_int()
        W = hostsim.hostsim_halfsize(k.to_bytes(32, "little"), c, d, ctypes.byref(neg))
        ci, di = int.from_bytes(c.raw, "little"), int.from_bytes(d.raw, "little")
        if neg.value:
            di = -di
        assert (ci - di * k) % (8 * L) == 0, k
        assert di % 2 == 1 and 0 < abs(di) < L, k
        assert 29 <= W <= 64 and max(ci.bit_length(), abs(di).bit_length()) <= 4 * W - 1, (k, W)
        if W == 64:
            assert (ci, di) == (k, 1)
        ws.append(W)
    rand = ws[14:]
    assert max(rand) <= 36 and sum(rand) / len(rand) < 32.8


def test_halfsize_torsion_keys(hostsim):
    """The half-size equation multiplies by d modulo the full group order 8L, so keys with a
    torsion component keep the reference's cofactorless decision: A = A0 + T (T of order 2, 4
    or 8) with R = [r]B - [k]T (valid) or R = [r]B (invalid unless [k]T = 0)."""
    rng = random.Random(9)
    small = E.small_order_points()
    pubs, sigs, msgs, exp = [], [], [], []
    for i in range(96):
        a = rng.randrange(1, E.L)
        T = small[i % 8]
        A = E.pt_add(E.pt_mul(a, E.BASE), T)
        pub = E.encode(A)
        m = rng.randbytes(40)
        r = rng.randrange(1, E.L)
        for mode in range(2):
            R0 = E.pt_mul(r, E.BASE)
            # k depends on R's bytes: pick R first, then S = r + k a (mod L)
            R = R0
            if mode == 0:
                # R = [r]B - [k]T requires k: iterate once with the k of the torsion-corrected R
                for _ in range(4):
                    Rb = E.encode(R)
                    k = int.from_bytes(hashlib.sha512(Rb + pub + m).digest(), "little") % E.L
                    R_new = E.pt_add(R0, E.pt_neg(E.pt_mul(k, T)))
                    if E.encode(R_new) == Rb:
                        break
                    R = R_new
            Rb = E.encode(R)
            k = int.from_bytes(hashlib.sha512(Rb + pub + m).digest(), "little") % E.L
            S = (r + k * a) % E.L
            pubs.append(pub)
            sigs.append(Rb + S.to_bytes(32, "little"))
            msgs.append(m)
            exp.append(1 if E.verify(pub, m, sigs[-1]) else 0)
    n = len(pubs)
    P = np.array([np.frombuffer(p, np.uint8) for p in pubs])
    Sg = np.array([np.frombuffer(s, np.uint8) for s in sigs])
    offs = np.zeros(n + 1, np.uint32)
    offs[1:] = np.cumsum([len(m) for m in msgs])
    M = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    out = _verify(hostsim, P, Sg, M, offs, "hs")
    assert (out == np.array(exp, np.uint8)).all()
    assert 0 < sum(exp) < n


def test_halfsize_fast_euclid_equals_reference_loop(hostsim):
    """verify_hs.h's two-steps-per-iteration Euclid phase (in-place, roles swapping) must stop at
    exactly the same remainder as the round-1 loop, so (c, d, W) are equal on every k — random k
    and the boundary values of the lattice test."""
    L = E.L
    rng = random.Random(11)
    ks = [0, 1, 2, 3, 8, 16, L - 1, L - 2, 2**127, 2**128 - 1, 2**128, 2**128 + 1, 2**160, 2**200,
          2**252 - 1, 5 * 2**128 + 3, (8 * L) // 3, (8 * L) // 5 + 1]
    ks += [rng.randrange(L) for _ in range(6000)]
    ks += [rng.randrange(2**129) for _ in range(300)] + [rng.randrange(2**170) for _ in range(300)]
    for k in ks:
        out = []
        for fn in (hostsim.hostsim_halfsize, hostsim.hostsim_halfsize_plain):
            c, d = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
            neg = ctypes.c_int()
            W = fn(k.to_bytes(32, "little"), c, d, ctypes.byref(neg))
            out.append((W, c.raw, d.raw, neg.value))
        assert out[0] == out[1], k


def test_halfsize_top_digit_and_wave_max(hostsim):
    """Random signatures through the half-size path (host build of verify_hs.h): with each lane's
    own tight W (x < 2^(4W): the top digit carries the recoding's overflow, digits up to 16, added
    as two table entries) and with W raised above it, as in a wave whose largest W exceeds the
    lane's; one flipped bit of S or of the message makes each invalid.  Decisions equal the
    oracle's C port; the tight count puts ~88 % of the lanes at 32 windows (the latency kernels'
    count, x < 2^(4W-1), ~40 %)."""
    rng = np.random.default_rng(17)
    n = 1536
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    offs = (np.arange(n + 1) * 110).astype(np.uint32)
    msgs = rng.integers(0, 256, int(offs[-1]) + 1, dtype=np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    pub = np.zeros((n, 32), np.uint8)
    hostsim.hostsim_sign_batch(_p(seeds), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(sig), _p(pub))
    sig[1::5, 40] ^= 4        # S changed
    msgs[offs[3:n:7]] ^= 1    # message changed
    exp = port.verify_batch(pub, sig, msgs, offs.astype(np.uint64), 8)
    assert 0 < exp.sum() < n
    wins = np.zeros(n, np.int32)
    for extra in (None, 1, 3):
        out = np.zeros(n, np.uint8)
        wmin = None if extra is None else _p(wins + extra)
        hostsim.hostsim_verify_batch_hs_w(_p(pub), _p(sig), _p(msgs), _p(offs), ctypes.c_size_t(n), _p(out),
                                          _p(wins) if extra is None else None, wmin)
        assert (out == exp).all(), (extra, np.nonzero(out != exp)[0][:8])
    assert wins.min() >= 29 and (wins == 32).sum() > n * 3 // 4 and wins.max() <= 34, np.bincount(wins)


def test_fused_carry_at_the_limb_extremes(hostsim):
    """fe_mul / fe_sq (3-sum inputs) and fe_sq2 (carried input) at the ends of the carried limb
    ranges (fe25519.h: even limbs [-2^25, 2^25), odd [0, 2^25), limb 1 [-2^16, 2^25 + 2^16), and
    fe_carry's odd [-2^24, 2^24]): the result is the product mod p and its limbs are carried."""
    P = E.P
    off = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    lo = [-(2**25) if i % 2 == 0 else -(2**24) for i in range(10)]
    hi = [2**25 - 1 if i % 2 == 0 else 2**25 - 1 for i in range(10)]
    lo[1], hi[1] = -(2**24) - 2**16, 2**25 + 2**16
    rng = random.Random(23)

    def val(c):
        return sum(x << o for x, o in zip(c, off))

    def carried():
        r = rng.random()
        if r < 0.3:
            return [lo[i] if rng.random() < 0.5 else hi[i] for i in range(10)]
        return [rng.randint(lo[i], hi[i]) for i in range(10)]

    def nsum(n):
        cs = [carried() for _ in range(n)]
        return [sum(c[i] for c in cs) for i in range(10)]

    cases = [([3 * hi[i] for i in range(10)], [3 * hi[i] for i in range(10)]),
             ([3 * lo[i] for i in range(10)], [3 * lo[i] for i in range(10)]),
             ([3 * hi[i] for i in range(10)], [3 * lo[i] for i in range(10)])]
    cases += [(nsum(3), nsum(3)) for _ in range(600)] + [(nsum(1), nsum(2)) for _ in range(300)]
    out = (ctypes.c_int32 * 10)()
    enc = ctypes.create_string_buffer(32)
    A = lambda c: (ctypes.c_int32 * 10)(*c)
    for a, b in cases:
        for op, exp, inputs_ok in ((0, val(a) * val(b), True), (1, val(a) ** 2, True),
                                   (2, 2 * val(a) ** 2, all(lo[i] <= a[i] <= hi[i] for i in range(10)))):
            if not inputs_ok:
                continue
            hostsim.hostsim_fe_raw(op, A(a), A(b), out, enc)
            assert int.from_bytes(enc.raw, "little") == exp % P, (op, a, b)
            u = list(out)
            for i in range(10):
                assert lo[i] <= u[i] <= hi[i] or (i % 2 == 1 and 0 <= u[i] < 2**25), (op, i, u[i])
    # fe_sq2 on carried inputs at the extremes
    for _ in range(400):
        a = carried()
        hostsim.hostsim_fe_raw(2, A(a), A(a), out, enc)
        assert int.from_bytes(enc.raw, "little") == 2 * val(a) ** 2 % P


@pytest.mark.parametrize("B", [10, 11, 12])
def test_radix_2_b_key_comb_digits(B):
    """The key-cached throughput kernel's signed radix-2^B digits of k (kernels.hip
    keyset_straus_ab24, kernels.h kCombA*; B = 12 by default), restated: W = floor(253 / B) windows;
    digit m < W - 1 is bits [Bm, Bm + B) + bit (Bm - 1) - 2^B * bit (Bm + B - 1), in
    [-2^(B-1), 2^(B-1)]; the top digit (m = W - 1) is every bit left + the bit below, unsigned, in
    [0, kCombATopMax] (B = 12: bits 240..252, [0, 4097]) — inside the comb's top window.  Sum of
    digit_m * 2^(Bm) = k for every k < L, including k in [2^252, L) where bit 252 is set."""
    L = 2**252 + 27742317777372353535851937790883648493
    W = 253 // B
    top_field = 253 - B * (W - 1)
    top_max = (1 << (top_field - 1)) + 1           # kernels.h kCombATopMax
    top_rows = ((top_max + 127) // 128) * 128 + 1  # kCombATopEntries
    mask = (1 << B) - 1
    rng = random.Random(11 + B)
    ks = [rng.randrange(L) for _ in range(3000)] + [L - 1, L - 2, 2**252, 2**252 + 12345, 0, 1, 2**241,
                                                     2**252 - 1, (2**253 - 1) % L, 2**240 - 1, 2**252 - 2**239]
    for k in ks:
        w = [(k >> (32 * i)) & 0xffffffff for i in range(8)]
        digits = []
        u = w[0] & mask
        digits.append(u - ((u >> (B - 1)) << B))
        for m in range(W - 1):
            below = (w[0] >> (B - 1)) & 1
            w = [((w[i] >> B) | (w[i + 1] << (32 - B))) & 0xffffffff for i in range(7)] + [w[7] >> B]
            last = m + 2 == W
            u = w[0] if last else w[0] & mask
            top = 0 if last else (u >> (B - 1)) << B
            digits.append(u + below - top)
        assert len(digits) == W
        h = 1 << (B - 1)
        assert all(-h <= d <= h for d in digits[:-1]) and 0 <= digits[-1] <= top_max < top_rows, (k, digits)
        assert sum(d << (B * m) for m, d in enumerate(digits)) == k, k
