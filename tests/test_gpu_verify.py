"""GPU parity: the gfx950 kernels through the C ABI vs the oracle (bit-exact decisions)."""
import hashlib
import os

import numpy as np
import pytest

from oracle import ed25519_go as E
from oracle import port

pytestmark = pytest.mark.gpu


def test_golden_vectors(generic_engine, golden):
    engine = generic_engine
    pubs = [bytes.fromhex(v["pub"]) for v in golden]
    msgs = [bytes.fromhex(v["msg"]) for v in golden]
    sigs = [bytes.fromhex(v["sig"]) for v in golden]
    out = engine.verify_batch(pubs, msgs, sigs)
    exp = np.array([v["valid"] for v in golden], np.uint8)
    bad = [golden[i]["class"] for i in np.nonzero(out != exp)[0]]
    assert not bad, bad
    assert exp.sum() > 600 and (exp == 0).sum() > 500


def _random_batch(n, seed, mlen=(0, 300)):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(mlen[0], mlen[1], n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    return rng, seeds, msgs, offs


def test_sign_kernel_matches_oracle(engine):
    rng, seeds, msgs, offs = _random_batch(3000, 1)
    sigs, pubs = engine.sign_arrays(seeds, msgs, offs.astype(np.uint32))
    esig, epub = port.sign_batch(seeds, msgs, offs, 8)
    assert (sigs == esig).all() and (pubs == epub).all()


def test_sign_kernel_privval_known_answer(engine):
    """The GPU signer's key derivation pinned to the reference's one fixed ed25519 datum
    (privval/msgs_test.go:62,85: GenPrivKeyFromSecret("it's a secret") -> 556a436f...c5fcf230),
    and a vote signed by it verifies on the GPU."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "privval_kat.json")) as f:
        kat = json.load(f)
    seed = np.frombuffer(hashlib.sha256(kat["secret_utf8"].encode()).digest(), np.uint8).reshape(1, 32)
    msg = np.frombuffer(b"privval vote" + bytes(16), np.uint8)
    offs = np.array([0, 12], np.uint32)
    sigs, pubs = engine.sign_arrays(seed, msg, offs)
    assert pubs[0].tobytes().hex() == kat["pubkey"]
    assert sigs[0].tobytes() == port.sign(seed[0].tobytes(), b"privval vote")
    out = engine.verify_arrays(pubs, sigs, msg, offs)
    assert out.tolist() == [1]


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 63, 64, 65, 255, 257, 1000])
def test_batch_sizes(generic_engine, n):
    engine = generic_engine
    rng, seeds, msgs, offs = _random_batch(n, 100 + n)
    sigs, pubs = port.sign_batch(seeds, msgs, offs, 8)
    sigs[::3, 5] ^= 0x10
    out = engine.verify_arrays(pubs, sigs, msgs, offs.astype(np.uint32))
    exp = port.verify_batch(pubs, sigs, msgs, offs, 8)
    assert (out == exp).all()


def test_c5_adversarial_mix(generic_engines):
    """C5: 1% invalid / non-canonical / small-order edge cases mixed into a valid batch (seed 0x5EED),
    through the throughput kernels (100k) and the latency kernels (the first 60k)."""
    engine = generic_engines["throughput"]
    n = 100_000
    rng, seeds, msgs, offs = _random_batch(n, 0x5EED, (100, 130))
    sigs, pubs = engine.sign_arrays(seeds, msgs, offs.astype(np.uint32))
    idx = rng.choice(n, n // 100, replace=False)
    small = [E.encode(p) for p in E.small_order_points()]
    for j, i in enumerate(idx):
        k = j % 6
        if k == 0:
            sigs[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)       # bit flip
        elif k == 1:
            S = int.from_bytes(sigs[i, 32:].tobytes(), "little") + E.L   # S + L
            sigs[i, 32:] = np.frombuffer(S.to_bytes(32, "little"), np.uint8)
        elif k == 2:
            pubs[i] = np.frombuffer(small[j % 8], np.uint8)               # small-order A
        elif k == 3:
            sigs[i, :32] = np.frombuffer(small[j % 8], np.uint8)          # small-order R
        elif k == 4:
            y = (int(rng.integers(0, 19)) + E.P).to_bytes(32, "little")   # non-canonical A (y >= p)
            pubs[i] = np.frombuffer(y, np.uint8)
        else:
            sigs[i, 31] ^= 0x80                                            # R sign flip
    out = engine.verify_arrays(pubs, sigs, msgs, offs.astype(np.uint32))
    exp = port.verify_batch(pubs, sigs, msgs, offs, 16)
    assert int((out != exp).sum()) == 0
    assert exp.sum() <= n - len(idx) + 16
    m = 60_000
    out = generic_engines["latency"].verify_arrays(pubs[:m], sigs[:m], msgs, offs[:m + 1].astype(np.uint32))
    assert int((out != exp[:m]).sum()) == 0


def test_full_size_property(engine):
    """BASELINE size (1,048,576): GPU-signed batch verifies all-valid; a bit flip in every
    signature flips every decision (size-independent property); a sample is checked by the port."""
    import torch
    from tmed.workload import c2_messages, c2_seeds
    n = 1 << 20
    seeds = c2_seeds(0, n)
    msgs, offs = c2_messages(0, n)
    dev = torch.device("cuda", 0)
    d_seed = torch.from_numpy(seeds).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch's fills before the engine's own stream (NULL = the context stream)
    engine.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n)
    engine.verify_device(d_pub, d_sig, d_msg, d_off, d_out, n)
    torch.cuda.synchronize()
    assert int(d_out.sum().item()) == n
    # the half-size hand-off is placed by window count (kernels.hip verify_prep_r_kernel): the
    # waves' loop length stays within ~0.1 window of the lanes' own mean (unplaced: ~0.7 above)
    lh, wh = engine.window_stats()
    ws = np.arange(65)
    assert int(lh.sum()) == n and int(wh.sum()) == n // 64 and int(lh[64]) == 0
    lane_mean, wave_mean = float((lh * ws).sum()) / n, float((wh * ws).sum()) / (n // 64)
    assert 32.0 < lane_mean < 33.0 and wave_mean - lane_mean < 0.3, (lane_mean, wave_mean)
    assert int(wh[32]) > n // 64 // 4
    d_sig[:, 40] ^= 1
    # (torch's flip runs on torch's stream; the engine's NULL stream is the context's own stream,
    # which is not ordered after it: the flip must be complete before the call)
    torch.cuda.synchronize()
    engine.verify_device(d_pub, d_sig, d_msg, d_off, d_out, n)
    torch.cuda.synchronize()
    assert int(d_out.sum().item()) == 0
    d_sig[:, 40] ^= 1
    torch.cuda.synchronize()
    m = 4096
    sl = slice(n - m, n)
    exp = port.verify_batch(d_pub[sl].cpu().numpy(), d_sig[sl].cpu().numpy(), msgs,
                            offs[n - m:].astype(np.uint64), 16)
    assert exp.all()
    assert d_sig[sl].cpu().numpy().tobytes() == port.sign_batch(seeds[n - m:], msgs, offs[n - m:].astype(np.uint64), 16)[0].tobytes()


def test_product_signbytes_match_oracle():
    from oracle.signbytes import vote_sign_bytes as ovsb
    from tmed.signbytes import vote_sign_bytes as pvsb
    rng = np.random.default_rng(4)
    for i in range(300):
        bid = None if i % 5 == 0 else (rng.bytes(32), int(rng.integers(0, 2**32)), rng.bytes(32))
        ts = (int(rng.integers(-2**40, 2**40)), int(rng.integers(0, 10**9)))
        h, r = int(rng.integers(0, 2**62)), int(rng.integers(-2**31, 2**31))
        cid = "c" * int(rng.integers(0, 51))
        flag = 3 if bid is None else 2
        assert pvsb(cid, h, r, bid, ts, flag) == ovsb(cid, 2, h, r, bid if flag == 2 else None, ts)


@pytest.fixture(params=["latency", "throughput"])
def keyset_engine(request, engine):
    """The default engine takes the latency kernels for key-cached batches up to TMED_LAT_MAX;
    a second engine with TMED_LAT_MAX=0 forces the throughput kernels on the same inputs."""
    if request.param == "latency":
        yield engine
        return
    from tmed import Engine
    old = os.environ.get("TMED_LAT_MAX")
    os.environ["TMED_LAT_MAX"] = "0"
    try:
        e = Engine(0)
    finally:
        if old is None:
            del os.environ["TMED_LAT_MAX"]
        else:
            os.environ["TMED_LAT_MAX"] = old
    yield e
    e.close()


def test_keyset_golden_and_random(keyset_engine, golden):
    """Key-cached comb path == generic path == oracle, on golden tuples grouped by key, through
    both the latency kernels (strict R decode + projective compare) and the throughput ones."""
    engine = keyset_engine
    vs = [v for v in golden if len(v["sig"]) == 128]
    keys = sorted({v["pub"] for v in vs})
    kidx = {k: i for i, k in enumerate(keys)}
    karr = np.array([np.frombuffer(bytes.fromhex(k), np.uint8) for k in keys])
    h = engine.keyset_load(karr)
    try:
        idx = np.array([kidx[v["pub"]] for v in vs], np.uint32)
        sigs = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs])
        ms = [bytes.fromhex(v["msg"]) for v in vs]
        offs = np.zeros(len(vs) + 1, np.uint32)
        offs[1:] = np.cumsum([len(m) for m in ms])
        msgs = np.frombuffer(b"".join(ms) + b"\0" * 16, np.uint8)
        out = engine.verify_keyset_arrays(h, idx, sigs, msgs, offs)
        exp = np.array([v["valid"] for v in vs], np.uint8)
        assert (out == exp).all(), [vs[i]["class"] for i in np.nonzero(out != exp)[0]][:10]
    finally:
        engine.keyset_free(h)
    # a 175-key set signing 20 commits' worth of votes, 1% corrupted
    rng, seeds, msgs, offs = _random_batch(175, 77, (110, 125))
    _, pubs = port.sign_batch(seeds, msgs, offs, 8)
    h = engine.keyset_load(pubs)
    try:
        n = 3500
        vi = rng.integers(0, 175, n).astype(np.uint32)
        lens = rng.integers(100, 160, n)
        o2 = np.zeros(n + 1, np.uint64)
        o2[1:] = np.cumsum(lens)
        m2 = rng.integers(0, 256, int(o2[-1]) + 16, dtype=np.uint8)
        sig2, _ = port.sign_batch(seeds[vi], m2, o2, 8)
        sig2[::97, 7] ^= 2
        out = engine.verify_keyset_arrays(h, vi, sig2, m2, o2.astype(np.uint32))
        exp = port.verify_batch(pubs[vi], sig2, m2, o2, 8)
        assert (out == exp).all() and exp.sum() == n - len(range(0, n, 97))
    finally:
        engine.keyset_free(h)


@pytest.mark.parametrize("lat_max", [0, 1 << 16])
def test_keyset_key_order_and_bad_indices(lat_max):
    """The throughput kernels visit a key-cached batch in key-grouped order (launch_key_order,
    n >= 4096): 20k signatures by 500 keys in random order must give the port's decisions at
    their own indices.  Through the device entry point (no host validation of val_idx) indices
    past the key set (500, 2^32 - 1) reject their signature instead of reading past the combs —
    in the throughput kernels (TMED_LAT_MAX=0) and in the latency kernels."""
    import torch
    from conftest import engine_with_env
    eng = engine_with_env(TMED_LAT_MAX=lat_max)
    rng, seeds, msgs, offs = _random_batch(500, 91, (110, 125))
    _, pubs = port.sign_batch(seeds, msgs, offs, 8)
    h = eng.keyset_load(pubs)
    try:
        n = 20_000
        vi = rng.integers(0, 500, n).astype(np.uint32)
        lens = rng.integers(100, 160, n)
        o2 = np.zeros(n + 1, np.uint64)
        o2[1:] = np.cumsum(lens)
        m2 = rng.integers(0, 256, int(o2[-1]) + 16, dtype=np.uint8)
        sig2, _ = port.sign_batch(seeds[vi], m2, o2, 16)
        sig2[::101, 9] ^= 4
        exp = port.verify_batch(pubs[vi], sig2, m2, o2, 16)
        out = eng.verify_keyset_arrays(h, vi, sig2, m2, o2.astype(np.uint32))
        assert int((out != exp).sum()) == 0
        bad = np.arange(7, n, 997)
        vi_bad = vi.copy()
        vi_bad[bad[::2]] = 500
        vi_bad[bad[1::2]] = 0xFFFFFFFF
        exp_bad = exp.copy()
        exp_bad[bad] = 0
        dev = torch.device("cuda", 0)
        d_vi = torch.from_numpy(vi_bad.view(np.int32)).to(dev)
        d_sig = torch.from_numpy(sig2).to(dev)
        d_msg = torch.from_numpy(m2).to(dev)
        d_off = torch.from_numpy(o2.astype(np.uint32).view(np.int32)).to(dev)
        d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        eng.verify_keyset_device(h, d_vi, d_sig, d_msg, d_off, d_out, n, 0)
        torch.cuda.synchronize(dev)
        assert int((d_out.cpu().numpy() != exp_bad).sum()) == 0
    finally:
        eng.keyset_free(h)
        eng.close()
