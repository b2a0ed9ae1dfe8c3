"""Key sets across comb chunks (kernels.h kKeyChunk*: 512 keys a chunk, each its own allocation,
the kernels reading a table of chunk bases).  An explicit key set of 1,100 keys (chunks of 512,
512 and 76 keys) is extended by 600 (the partial chunk replaced by a larger one, its built keys
copied over; one new chunk).  Batches through the throughput kernels (both combs) and the latency
kernels, with indexes over every key, equal the port oracle before and after; comb rows read back
at the chunk edges equal j * R^w * (-A)."""
import numpy as np
import pytest

from oracle import port
from test_gpu_btables import _limbs_to_int, _niels

pytestmark = pytest.mark.gpu


def _keys(n, seed):
    seeds = np.random.default_rng(seed).integers(0, 256, (n, 32), dtype=np.uint8)
    offs = np.arange(n + 1, dtype=np.uint64) * 8
    msgs = np.zeros(8 * n + 16, np.uint8)
    _, pubs = port.sign_batch(seeds, msgs, offs, 8)
    return seeds, pubs


def _batch(seeds, pubs, nkeys, n, seed):
    rng = np.random.default_rng(seed)
    vi = rng.integers(0, nkeys, n).astype(np.uint32)
    vi[:4] = [0, nkeys - 1, min(511, nkeys - 1), min(512, nkeys - 1)]
    lens = rng.integers(100, 140, n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, _ = port.sign_batch(seeds[vi], msgs, offs, 8)
    sigs[::37, 5] ^= 2
    exp = port.verify_batch(pubs[vi], sigs, msgs, offs, 8)
    return vi, sigs, msgs, offs.astype(np.uint32), exp


def _rows_match(eng, h, pubs, keys, bits_list):
    from oracle import ed25519_go as E
    for key in keys:
        pt = E.decode(bytes(pubs[key]))
        assert pt is not None
        base = E.pt_neg(pt)
        for bits in bits_list:
            W = 32 if bits == 8 else 253 // bits
            top = 128 if bits == 8 else 4224
            for w, j in ((0, 1), (1, 9), (W - 1, top)):
                row = eng.keyset_comb_entry(h, key, bits, w, j)
                got = tuple(_limbs_to_int(row[10 * c:10 * c + 10]) % E.P for c in range(3))
                assert got == _niels(E.pt_mul(j * (1 << (bits * w)), base)), (key, bits, w, j)


def test_key_set_across_chunks(engine):
    seeds, pubs = _keys(1700, 77)
    h = engine.keyset_load(pubs[:1100])
    try:
        big = _batch(seeds, pubs, 1100, 40000, 1)
        assert (engine.verify_keyset_arrays(h, *big[:4]) == big[4]).all()  # throughput: builds the 2^12 comb
        assert engine.keyset_a_window_bits(h) == 12
        small = _batch(seeds, pubs, 1100, 700, 2)
        assert (engine.verify_keyset_arrays(h, *small[:4]) == small[4]).all()  # latency kernels
        _rows_match(engine, h, pubs, (511, 512, 1023, 1024, 1099), (8, 12))
        assert engine.keyset_extend(h, pubs[1100:]) == 1100
        big2 = _batch(seeds, pubs, 1700, 40000, 3)
        assert (engine.verify_keyset_arrays(h, *big2[:4]) == big2[4]).all()  # the 2^12 comb extended
        assert engine.keyset_a_window_bits(h) == 12
        small2 = _batch(seeds, pubs, 1700, 700, 4)
        assert (engine.verify_keyset_arrays(h, *small2[:4]) == small2[4]).all()
        _rows_match(engine, h, pubs, (1024, 1099, 1100, 1535, 1536, 1699), (8, 12))
    finally:
        engine.keyset_free(h)


def test_key_set_table_growth(engine):
    """An explicit set's chunk tables are sized to its keys (8 entries per comb for up to 4,096 keys,
    not the pool's 32,768): extending a 600-key set to 4,700 keys (10 chunks) moves both tables into
    larger ones, the radix-2^12 half at its new offset.  Batches over every key through both combs
    and the latency kernels equal the port before and after; comb rows at the far chunks read back."""
    seeds, pubs = _keys(4700, 78)
    h = engine.keyset_load(pubs[:600])
    try:
        big = _batch(seeds, pubs, 600, 30000, 11)  # > TMED_LAT_MAX (24,576): the throughput kernels
        assert (engine.verify_keyset_arrays(h, *big[:4]) == big[4]).all()
        assert engine.keyset_a_window_bits(h) == 12
        assert engine.keyset_extend(h, pubs[600:]) == 600
        big2 = _batch(seeds, pubs, 4700, 40000, 12)
        assert (engine.verify_keyset_arrays(h, *big2[:4]) == big2[4]).all()
        assert engine.keyset_a_window_bits(h) == 12
        small2 = _batch(seeds, pubs, 4700, 700, 13)
        assert (engine.verify_keyset_arrays(h, *small2[:4]) == small2[4]).all()
        _rows_match(engine, h, pubs, (599, 4095, 4096, 4699), (8, 12))
    finally:
        engine.keyset_free(h)


def test_full_size_keyed_property(engine):
    """BASELINE's key-cached C2 variant at full size: 2^20 GPU-signed signatures by 10,000 keys (20
    comb chunks, 64 GB of combs) through the throughput kernels on the radix-2^12 comb: every
    decision valid; a bit flipped in every signature flips every decision (size-independent); a
    4,096-signature sample equals the port; an index past the set rejects."""
    import torch
    from tmed.workload import c2_messages, seeds_from_tag
    n, nk = 1 << 20, 10_000
    kseeds = seeds_from_tag(b"tmed-c2k-key", 0, nk)
    val_idx = np.random.default_rng(7).integers(0, nk, n).astype(np.uint32)
    msgs, offs = c2_messages(0, n)
    dev = torch.device("cuda", 0)
    d_seed = torch.from_numpy(kseeds[val_idx]).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch's fills before the engine's own stream (NULL = the context stream)
    engine.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n)
    torch.cuda.synchronize()
    pubs = np.zeros((nk, 32), np.uint8)
    pubs[val_idx] = d_pub.cpu().numpy()
    del d_seed, d_pub
    h = engine.keyset_load(pubs)
    try:
        d_vi = torch.from_numpy(val_idx.view(np.int32)).to(dev)
        engine.verify_keyset_device(h, d_vi, d_sig, d_msg, d_off, d_out, n)
        torch.cuda.synchronize()
        assert engine.keyset_a_window_bits(h) == 12
        assert int(d_out.sum().item()) == n
        d_sig[:, 40] ^= 1
        torch.cuda.synchronize()  # torch's flip before the engine's own (NULL = context) stream reads it
        engine.verify_keyset_device(h, d_vi, d_sig, d_msg, d_off, d_out, n)
        torch.cuda.synchronize()
        assert int(d_out.sum().item()) == 0
        d_sig[:, 40] ^= 1
        d_vi[12345] = nk  # past the set: rejected, the rest unchanged
        torch.cuda.synchronize()
        engine.verify_keyset_device(h, d_vi, d_sig, d_msg, d_off, d_out, n)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        assert out[12345] == 0 and int(out.sum()) == n - 1
        m = 4096
        sl = slice(n - m, n)
        exp = port.verify_batch(pubs[val_idx[sl]], d_sig[sl].cpu().numpy(), msgs, offs[n - m:].astype(np.uint64), 16)
        assert exp.all() and out[sl].all()
    finally:
        engine.keyset_free(h)


@pytest.mark.parametrize("fail_at,what", [(5, "load"), (7, "comba chunk"), (8, "comba scratch")])
def test_key_set_allocation_failures(fail_at, what, engine):
    """Out of memory at each step of a key set's life (TMED_TEST_FAIL_KS_ALLOC=n: the context's n-th
    key-set allocation fails; a 700-key set allocates its table, encodings, flags and comb chunks
    1-5 at load, then the radix-2^12 comb's chunks 6-7 and build scratch 8 at its first throughput
    batch).  A failed load reports ENOMEM and leaves nothing behind (the next load works); a failed
    radix-2^12 comb leaves the set on its radix-256 comb.  Decisions equal the port either way."""
    from conftest import engine_with_env
    from tmed._native import TmedError
    eng = engine_with_env(TMED_TEST_FAIL_KS_ALLOC=fail_at)
    try:
        seeds, pubs = _keys(700, 31)
        if what == "load":
            with pytest.raises(TmedError):
                eng.keyset_load(pubs)
        h = eng.keyset_load(pubs)
        try:
            big = _batch(seeds, pubs, 700, 30000, 5)
            assert (eng.verify_keyset_arrays(h, *big[:4]) == big[4]).all()
            assert eng.keyset_a_window_bits(h) == (12 if what == "load" else 8)
            small = _batch(seeds, pubs, 700, 500, 6)
            assert (eng.verify_keyset_arrays(h, *small[:4]) == small[4]).all()
            assert (eng.verify_keyset_arrays(h, *big[:4]) == big[4]).all()
        finally:
            eng.keyset_free(h)
    finally:
        eng.close()


def test_pool_append_failure_stays_generic(engine):
    """The key-set cache's pool runs out of memory at its first append (TMED_TEST_FAIL_KS_ALLOC=4:
    its first comb chunk): that window runs on the generic kernels with the same outcomes, nothing
    is pooled, and the next window of the set builds its keys and is keyed."""
    from conftest import engine_with_env
    from test_gpu_keycache import _bs_window, _delta
    import tmed.types as T
    eng = engine_with_env(TMED_KEYCACHE=1, TMED_TEST_FAIL_KS_ALLOC=4)
    try:
        eng.keycache_config(True, 8 << 30)
        w = _bs_window(eng, b"kc-oom", nv=64, nb=4096)
        ref = T.BlocksyncWindow(*w)
        ref.run(engine, 128)
        for keyed in (0, 1):
            s0 = eng.keycache_stats()
            got = T.BlocksyncWindow(*w)
            got.run(eng, 128)
            d = _delta(s0, eng.keycache_stats())
            assert (got.codes() == ref.codes()).all() and (got.verified() == ref.verified()).all()
            assert d["keyed_sets"] == keyed and d["keys_appended"] == 64 * keyed, d
        assert eng.keycache_stats()["pool_keys"] == 64
    finally:
        eng.close()
