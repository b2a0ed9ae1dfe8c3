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
