"""GPU: the fixed-base tables of B.  The default path runs on the radix-2^26 tables
(8.6 GB, shared per device) and the key-cached throughput path on the radix-2^24 comb (11.8 GB,
acquired at the first key-set load); TMED_B26=0 / TMED_B24=0 keep both on the context's radix-2^16
comb.  Same decisions either way: the golden vectors through the throughput kernels of both
configurations against the oracle's expected answers."""
import numpy as np
import pytest

from conftest import engine_with_env

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def radix_engines():
    es = {"default": engine_with_env(TMED_GLAT_MAX=0, TMED_LAT_MAX=0),
          "radix16": engine_with_env(TMED_GLAT_MAX=0, TMED_LAT_MAX=0, TMED_B26=0, TMED_B24=0),
          "a8": engine_with_env(TMED_GLAT_MAX=0, TMED_LAT_MAX=0, TMED_KS_ACOMB=0)}
    yield es
    for e in es.values():
        e.close()


def _golden_arrays(golden):
    vs = [v for v in golden if len(v["sig"]) == 128]
    keys = sorted({v["pub"] for v in vs})
    kidx = {k: i for i, k in enumerate(keys)}
    karr = np.array([np.frombuffer(bytes.fromhex(k), np.uint8) for k in keys])
    idx = np.array([kidx[v["pub"]] for v in vs], np.uint32)
    sigs = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs])
    ms = [bytes.fromhex(v["msg"]) for v in vs]
    offs = np.zeros(len(vs) + 1, np.uint32)
    offs[1:] = np.cumsum([len(m) for m in ms])
    msgs = np.frombuffer(b"".join(ms) + b"\0" * 16, np.uint8)
    exp = np.array([v["valid"] for v in vs], np.uint8)
    return vs, karr, idx, sigs, msgs, offs, exp


@pytest.mark.parametrize("cfg,b_bits,ks_bits,a_bits", [("default", 26, 24, 12), ("radix16", 16, 16, 8),
                                                       ("a8", 26, 24, 8)])
def test_b_window_radix_and_decisions(radix_engines, golden, cfg, b_bits, ks_bits, a_bits):
    """...and the key-cached throughput kernel's -A comb: radix 2^12 (built at the key set's first
    throughput batch) by default, the radix-256 comb with TMED_KS_ACOMB=0 or without the radix-2^24 B
    comb."""
    eng = radix_engines[cfg]
    assert eng.b_window_bits() == b_bits
    vs, karr, idx, sigs, msgs, offs, exp = _golden_arrays(golden)
    out = eng.verify_batch([bytes.fromhex(v["pub"]) for v in vs], [bytes.fromhex(v["msg"]) for v in vs],
                           [bytes.fromhex(v["sig"]) for v in vs])
    assert (out == exp).all(), [vs[i]["class"] for i in np.nonzero(out != exp)[0]][:10]
    h = eng.keyset_load(karr)
    try:
        assert eng.keyset_b_window_bits() == ks_bits
        assert eng.keyset_a_window_bits(h) == 8  # before the first throughput batch
        out = eng.verify_keyset_arrays(h, idx, sigs, msgs, offs)
        assert (out == exp).all(), [vs[i]["class"] for i in np.nonzero(out != exp)[0]][:10]
        assert eng.keyset_a_window_bits(h) == a_bits
        out = eng.verify_keyset_arrays(h, idx, sigs, msgs, offs)
        assert (out == exp).all(), [vs[i]["class"] for i in np.nonzero(out != exp)[0]][:10]
    finally:
        eng.keyset_free(h)


def _limbs_to_int(v):
    """30 int32 limbs of radix 2^25.5 (limb i weighs 2^ceil(25.5 i)) -> an integer (mod p)."""
    off = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
    return sum(int(x) << o for x, o in zip(v, off))


def _niels(pt):
    from oracle import ed25519_go as E
    x, y, z, _ = pt
    zi = pow(z, E.P - 2, E.P)
    x, y = x * zi % E.P, y * zi % E.P
    return ((y + x) % E.P, (y - x) % E.P, 2 * E.D * x * y % E.P)


def test_key_comb_rows_equal_the_oracle(radix_engines, golden):
    """Both key combs, read back row by row (tmed_keyset_comb_entry) and compared with
    j * R^w * (-A) from the oracle: the radix-256 comb every key set holds (R = 256) and the
    throughput comb (R = 2^12, built at the set's first throughput batch), at the edges of the
    kernels' runs of 8 entries (comb_fill_run: one double-and-add, then additions, one batched
    inversion per run), the windows' last entries and the top window's range, for keys that decode
    and keys that do not (their base is the identity, every row (1, 1, 0))."""
    from oracle import ed25519_go as E
    eng = radix_engines["default"]
    vs, karr, idx, sigs, msgs, offs, exp = _golden_arrays(golden)
    pts = [E.decode(bytes(k)) for k in karr]
    good = [i for i, p in enumerate(pts) if p is not None][:3]
    bad = [i for i, p in enumerate(pts) if p is None][:1]
    h = eng.keyset_load(karr)
    try:
        eng.verify_keyset_arrays(h, idx, sigs, msgs, offs)  # the first throughput batch builds the 2^12 comb
        B = eng.keyset_a_window_bits(h)
        assert B == 12
        W = 253 // B
        cases = [(8, w, j) for w in (0, 1, 17, 31) for j in (0, 1, 2, 8, 9, 16, 17, 64, 127, 128)]
        cases += [(B, w, j) for w in (0, 1, 11, W - 2) for j in (0, 1, 7, 8, 9, 10, 1023, 1024, 2041, 2047, 2048)]
        cases += [(B, W - 1, j) for j in (0, 1, 8, 9, 2048, 2049, 4096, 4097, 4217, 4224)]
        for key in good + bad:
            for bits, w, j in cases:
                row = eng.keyset_comb_entry(h, key, bits, w, j)
                got = tuple(_limbs_to_int(row[10 * c:10 * c + 10]) % E.P for c in range(3))
                if pts[key] is None or j == 0:
                    assert got == (1, 1, 0), (key, bits, w, j)
                    continue
                base = E.pt_neg(pts[key])
                want = _niels(E.pt_mul(j * (1 << ((8 if bits == 8 else bits) * w)), base))
                assert got == want, (key, bits, w, j)
        with pytest.raises(Exception):
            eng.keyset_comb_entry(h, 0, B, W - 1, 4225)  # past the top window
    finally:
        eng.keyset_free(h)
