"""GPU parity of the generic main-kernel variants other than the context default, each on
its own context (TMED_MAIN_WAVES is read by tmed_init): the half-size-scalar path
(verify_hs.h, variant 6) and the full-length Straus path with the batched finish
(variant 5).  Decisions must equal the oracle's bit for bit on every golden class, on
random batches with flipped bits, and on the C5 adversarial mix."""
import os

import numpy as np
import pytest

from oracle import ed25519_go as E
from oracle import port

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[5, 6])
def vengine(request):
    from tmed import Engine
    old = os.environ.get("TMED_MAIN_WAVES")
    os.environ["TMED_MAIN_WAVES"] = str(request.param)
    try:
        e = Engine(0)
    finally:
        if old is None:
            del os.environ["TMED_MAIN_WAVES"]
        else:
            os.environ["TMED_MAIN_WAVES"] = old
    yield e
    e.close()


def test_golden(vengine, golden):
    pubs = [bytes.fromhex(v["pub"]) for v in golden]
    msgs = [bytes.fromhex(v["msg"]) for v in golden]
    sigs = [bytes.fromhex(v["sig"]) for v in golden]
    out = vengine.verify_batch(pubs, msgs, sigs)
    exp = np.array([v["valid"] for v in golden], np.uint8)
    bad = [golden[i]["class"] for i in np.nonzero(out != exp)[0]]
    assert not bad, bad


@pytest.mark.parametrize("n", [1, 65, 1000, 20000])
def test_random_flips(vengine, n):
    rng = np.random.default_rng(7 + n)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(0, 300, n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = vengine.sign_arrays(seeds, msgs, offs.astype(np.uint32))
    sigs[::3, rng.integers(0, 64)] ^= 0x04
    out = vengine.verify_arrays(pubs, sigs, msgs, offs.astype(np.uint32))
    exp = port.verify_batch(pubs, sigs, msgs, offs, 16)
    assert int((out != exp).sum()) == 0


def test_c5_mix(vengine):
    n = 50_000
    rng = np.random.default_rng(0x5EED)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    offs = (np.arange(n + 1) * 115).astype(np.uint64)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = vengine.sign_arrays(seeds, msgs, offs.astype(np.uint32))
    small = [E.encode(p) for p in E.small_order_points()]
    idx = rng.choice(n, n // 50, replace=False)
    for j, i in enumerate(idx):
        k = j % 5
        if k == 0:
            sigs[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
        elif k == 1:
            pubs[i] = np.frombuffer(small[j % 8], np.uint8)
        elif k == 2:
            sigs[i, :32] = np.frombuffer(small[j % 8], np.uint8)
        elif k == 3:
            pubs[i] = np.frombuffer((int(rng.integers(0, 19)) + E.P).to_bytes(32, "little"), np.uint8)
        else:
            sigs[i, 31] ^= 0x80
    out = vengine.verify_arrays(pubs, sigs, msgs, offs.astype(np.uint32))
    exp = port.verify_batch(pubs, sigs, msgs, offs, 16)
    assert int((out != exp).sum()) == 0


@pytest.mark.parametrize("slots,chunk", [("1000", None), ("300", "100")])
def test_odd_slab_and_chunk_sizes(slots, chunk):
    """TMED_SLAB_SLOTS / TMED_CHUNK that are not multiples of the 256-lane block: the
    context rounds them up, so every lane of every launched block owns a slab slot and a batch
    larger than the slab runs as several chunks with decisions equal to the oracle.  TMED_GLAT_MAX=0
    sends the batch through the throughput kernels (prep / prep_r / main chunks), not the latency
    kernels that take small batches by default."""
    from tmed import Engine
    saved = {k: os.environ.get(k) for k in ("TMED_SLAB_SLOTS", "TMED_CHUNK", "TMED_GLAT_MAX")}
    os.environ["TMED_GLAT_MAX"] = "0"
    os.environ["TMED_SLAB_SLOTS"] = slots
    if chunk:
        os.environ["TMED_CHUNK"] = chunk
    try:
        e = Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        n = 2600
        rng = np.random.default_rng(99)
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        offs = (np.arange(n + 1) * 114).astype(np.uint64)
        msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
        sigs, pubs = e.sign_arrays(seeds, msgs, offs.astype(np.uint32))
        sigs[::7, 40] ^= 0x01
        out = e.verify_arrays(pubs, sigs, msgs, offs.astype(np.uint32))
        exp = port.verify_batch(pubs, sigs, msgs, offs, 16)
        assert int((out != exp).sum()) == 0 and exp.sum() == n - len(range(0, n, 7))
    finally:
        e.close()


def test_partial_chunk_after_full_slab():
    """A full-slab batch, then batches of slab_slots - k: the lanes past count in the
    last wave of verify_main_hs_kernel sit on hand-off positions that still hold the previous
    batch's recodings; they must run on zero digits (HsDigitsDev.active) and the decisions of the
    short batch must equal the oracle's."""
    from tmed import Engine
    saved = {k: os.environ.get(k) for k in ("TMED_SLAB_SLOTS", "TMED_GLAT_MAX")}
    os.environ["TMED_GLAT_MAX"] = "0"
    os.environ["TMED_SLAB_SLOTS"] = "2048"
    try:
        e = Engine(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        n = 2048
        rng = np.random.default_rng(123)
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        offs = (np.arange(n + 1) * 114).astype(np.uint64)
        msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
        sigs, pubs = e.sign_arrays(seeds, msgs, offs.astype(np.uint32))
        sigs[::5, 33] ^= 0x10
        exp = port.verify_batch(pubs, sigs, msgs, offs, 16)
        for m in (n, n - 1, n - 63, n - 200, n - 255, n, 1800):
            out = e.verify_arrays(pubs[:m], sigs[:m], msgs, offs[: m + 1].astype(np.uint32))
            assert int((out != exp[:m]).sum()) == 0, m
    finally:
        e.close()
