"""One context shared by concurrent callers (SURVEY.md §8b "Threading": the blocksync
goroutine, the light client, the evidence pool and RPC may all verify at once).  Several
host threads drive every entry point of ONE engine at the same time — host-buffer batches
(generic and key-cached, latency and throughput sizes), the commit seam, the Merkle hashes,
and device-pointer batches on their own HIP streams sharing the context's scratch — and
every result must equal the one computed serially.  (ctypes releases the GIL for the C
calls, so the calls really overlap.)"""
import threading

import numpy as np
import pytest

from oracle import port

pytestmark = pytest.mark.gpu


def _batch(n, seed):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(90, 170, n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = port.sign_batch(seeds, msgs, offs, 8)
    sigs[::53, 40] ^= 1
    return pubs, sigs, msgs, offs.astype(np.uint32)


def test_concurrent_callers_share_one_context(engine):
    import torch
    from commit_cases import oracle_result, pbid, same, scenarios
    import tmed.types as T
    from tmed import merkle as TM

    pubs, sigs, msgs, offs = _batch(6000, 11)
    exp_generic = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 8)
    kpubs = pubs[:200].copy()
    ks = engine.keyset_load(kpubs)
    rng = np.random.default_rng(3)
    vi = rng.integers(0, 200, 30000).astype(np.uint32)
    kl = rng.integers(100, 140, vi.size)
    ko = np.zeros(vi.size + 1, np.uint64)
    ko[1:] = np.cumsum(kl)
    km = rng.integers(0, 256, int(ko[-1]) + 16, dtype=np.uint8)
    seeds = np.random.default_rng(11).integers(0, 256, (6000, 32), dtype=np.uint8)[:200]
    ksig, _ = port.sign_batch(seeds[vi], km, ko, 8)
    ksig[::71, 3] ^= 4
    exp_keyed = port.verify_batch(kpubs[vi], ksig, km, ko, 8)
    ko32 = ko.astype(np.uint32)
    reqs, exp_commits = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=21, count=40):
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
        exp_commits.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
    S, V = 300, 175
    vpub = np.random.default_rng(5).integers(0, 256, (S * V, 32), dtype=np.uint8)
    vpow = np.full(S * V, 10, np.int64)
    voff = (np.arange(S + 1) * V).astype(np.uint32)
    exp_vh = TM.valset_hashes_arrays(engine, vpub, vpow, voff).copy()

    dev = torch.device("cuda", 0)
    d_pub = torch.from_numpy(pubs).to(dev)
    d_sig = torch.from_numpy(sigs).to(dev)
    d_msg = torch.from_numpy(msgs).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    torch.cuda.synchronize(dev)

    errors = []

    def run(name, fn, reps):
        try:
            for _ in range(reps):
                fn()
        except Exception as e:  # reported below with the failing caller's name
            errors.append("%s: %r" % (name, e))

    def generic():
        assert (engine.verify_arrays(pubs, sigs, msgs, offs) == exp_generic).all()

    def keyed_small():
        out = engine.verify_keyset_arrays(ks, vi[:1500], ksig[:1500], km, ko32[:1501])
        assert (out == exp_keyed[:1500]).all()

    def keyed_large():
        assert (engine.verify_keyset_arrays(ks, vi, ksig, km, ko32) == exp_keyed).all()

    def commits():
        got = T.verify_commits(engine, reqs)
        assert all(same(g, e) for g, e in zip(got, exp_commits))

    def merkle():
        assert (TM.valset_hashes_arrays(engine, vpub, vpow, voff) == exp_vh).all()

    def device_stream():
        st = torch.cuda.Stream(dev)
        d_out = torch.zeros(pubs.shape[0], dtype=torch.uint8, device=dev)
        st.wait_stream(torch.cuda.current_stream(dev))  # the zero fill (torch's stream) before the engine's work on st
        engine.verify_device(d_pub, d_sig, d_msg, d_off, d_out, pubs.shape[0], st.cuda_stream)
        st.synchronize()
        assert (d_out.cpu().numpy() == exp_generic).all()

    try:
        jobs = [("generic", generic, 4), ("keyed_small", keyed_small, 8), ("keyed_large", keyed_large, 3),
                ("commits", commits, 4), ("merkle", merkle, 6), ("device_a", device_stream, 4),
                ("device_b", device_stream, 4)]
        ths = [threading.Thread(target=run, args=j) for j in jobs]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=110)
        assert not any(t.is_alive() for t in ths), "a caller did not finish"
        assert not errors, errors
    finally:
        engine.keyset_free(ks)
