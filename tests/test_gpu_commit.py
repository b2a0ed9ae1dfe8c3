"""GPU commit seam: tmed_verify_commits (C++ plan/replay + gfx950 batch) vs the reference loops."""
import pytest

from commit_cases import oracle_result, pbid, same, scenarios
import tmed.types as T

pytestmark = pytest.mark.gpu


def test_seam_matches_reference_loops_gpu(engine):
    reqs, exp = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=2, count=120):
        exp.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    got = T.verify_commits(engine, reqs)
    bad = [(q, str(g), str(e)) for q, (g, e) in enumerate(zip(got, exp)) if not same(g, e)]
    assert not bad, bad[:5]
    for q in range(0, len(reqs), 7):
        assert same(T.verify_commits(engine, [reqs[q]])[0], exp[q])


def test_pipelined_seam_gpu(engine):
    """Large tmed_verify_commits calls go through the two-slot pipeline (batches planned and
    staged while the previous batch runs); TMED_PIPE_SIGS=64 forces many tiny batches, and the
    pipelined path must reproduce the reference loops on every scenario, batch boundaries
    included."""
    import os
    reqs, exp = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=3, count=90):
        exp.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    os.environ["TMED_PIPE_SIGS"] = "64"
    try:
        got = T.verify_commits(engine, reqs)
    finally:
        del os.environ["TMED_PIPE_SIGS"]
    bad = [(q, str(g), str(e)) for q, (g, e) in enumerate(zip(got, exp)) if not same(g, e)]
    assert not bad, bad[:5]


def test_oversize_chain_ids_and_mixed_key_sets_gpu(engine):
    """One seam call mixing generic requests, requests on several key sets (one launch group
    per key set) and chain IDs too long for the device sign-bytes template (host-assembled
    fallback; VerifyCommit itself does not bound the chain ID) — every decision and error
    equal to the reference loops."""
    import numpy as np
    long_chain = "c" * 200
    reqs, exp, handles = [], [], []
    try:
        for k, (mode, vs, pv, chain, bid, h, cm, pc, num, den) in enumerate(
                scenarios(seed=11, count=48, chains=("test_chain_id", long_chain))):
            if k % 3 == 1:  # key-cached: a key set per request (keys in set order)
                pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators])
                pv.keyset = engine.keyset_load(pubs)
                pv.keyset_index = np.arange(len(pubs), dtype=np.uint32)
                handles.append(pv.keyset)
            exp.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
            reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
        got = T.verify_commits(engine, reqs)
        bad = [(q, str(g), str(e)) for q, (g, e) in enumerate(zip(got, exp)) if not same(g, e)]
        assert not bad, bad[:5]
        assert any(r[2] == long_chain for r in reqs) and handles
    finally:
        for hnd in handles:
            engine.keyset_free(hnd)


def test_multi_context_sharding_gpu(engine):
    """tmed_verify_commits_multi / tmed_blocksync_verify_multi: requests sharded over several
    contexts in one process (here three contexts on the one GPU of the test box; on a node,
    one per GPU) give exactly the single-context results, key-set handles included."""
    import numpy as np
    from tmed import Engine
    engines = [Engine(0) for _ in range(3)]  # fresh contexts: key-set handles count up in step
    try:
        reqs, exp = [], []
        for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=13, count=70):
            exp.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
            reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
        got = T.verify_commits(engines, reqs)
        bad = [(q, str(g), str(e)) for q, (g, e) in enumerate(zip(got, exp)) if not same(g, e)]
        assert not bad, bad[:5]
        # blocksync window over one key set, loaded on every context (same handle everywhere)
        from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of
        from commit_cases import to_product
        vs, seeds = make_valset([seed_of("mc", i) for i in range(7)], [10] * 7)
        blocks, bids, heights, wexp = [], [], [], []
        for h in range(9):
            bid = make_block_id("mc%d" % h)
            cm = make_commit(vs, seeds, "mc-chain", 10 + h, 0, bid)
            if h == 4:
                resign(cm, 1, seeds[1], "bad")
            wexp.append(oracle_result(T.MODE_LIGHT, vs, "mc-chain", bid, 10 + h, cm, 0, 0))
            blocks.append(to_product(vs, cm)[1])
            bids.append(pbid(bid))
            heights.append(10 + h)
        pv = to_product(vs, make_commit(vs, seeds, "mc-chain", 1, 0, make_block_id("y")))[0]
        pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators])
        hs = [e.keyset_load(pubs) for e in engines]
        assert len(set(hs)) == 1
        pv.keyset = hs[0]
        try:
            w = T.BlocksyncWindow(pv, "mc-chain", bids, heights, blocks)
            w.run(engines, 2)
            assert all(same(g, e) for g, e in zip(w.errors(), wexp))
        finally:
            for e, hnd in zip(engines, hs):
                e.keyset_free(hnd)
    finally:
        for e in engines:
            e.close()


def test_index_sliced_commit_gpu(engine):
    """§8e latency mode on one rank: the slice verifier runs on the GPU (tmed_verify_batch) and
    the first-failure replay must give the reference loop's exact error."""
    from tmed.dist import verify_commit_sliced
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=5, count=40):
        e = oracle_result(mode, vs, chain, bid, h, cm, num, den)
        got, _ = verify_commit_sliced(engine, (mode, pv, chain, pbid(bid), h, pc, num, den), 0, 1)
        assert same(got, e), (str(got), str(e))


def test_reference_cases_gpu(engine):
    """types/validator_set_test.go:746-815 through the GPU seam."""
    from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("g", i) for i in range(4)], [10] * 4)
    bid = make_block_id("g")
    cm = make_commit(vs, seeds, "test_chain_id", 3, 0, bid)
    resign(cm, 3, seeds[3], "CentaurusA")
    pv, pc = to_product(vs, cm)
    assert "wrong signature (#3)" in str(pv.verify_commit(engine, "test_chain_id", pbid(bid), 3, pc))
    assert pv.verify_commit_light(engine, "test_chain_id", pbid(bid), 3, pc) is None
    cm2 = make_commit(vs, seeds, "test_chain_id", 3, 0, bid)
    resign(cm2, 2, seeds[2], "CentaurusA")
    pv, pc2 = to_product(vs, cm2)
    assert pv.verify_commit_light_trusting(engine, "test_chain_id", pc2, 1, 3) is None


def test_keyset_seam_and_packed_commits(engine):
    """Key-cached seam (global key set + per-valset index) and PackedCommit == reference loops."""
    import numpy as np
    from oracle import commit as C
    from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("ks", i) for i in range(12)], [10] * 11 + [30])
    bid = make_block_id("ks")
    cms = []
    for h in range(6):
        cm = make_commit(vs, seeds, "kc", 100 + h, 0, bid)
        if h % 2:
            resign(cm, h, seeds[h], "bad")
        cms.append(cm)
    pv, _ = to_product(vs, cms[0])
    pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators])
    # key set holds the keys in reverse order: exercise keyset_index
    ks = engine.keyset_load(pubs[::-1].copy())
    pv.keyset = ks
    pv.keyset_index = np.arange(len(pubs) - 1, -1, -1).astype(np.uint32)
    try:
        reqs, exp = [], []
        for cm in cms:
            _, pc = to_product(vs, cm)
            packed = T.PackedCommit(pc.height, pc.round, pc.block_id,
                                    np.array([s.flag for s in pc.signatures], np.uint8),
                                    np.array([np.frombuffer(s.address, np.uint8) for s in pc.signatures]),
                                    np.array([s.timestamp[0] for s in pc.signatures], np.int64),
                                    np.array([s.timestamp[1] for s in pc.signatures], np.int32),
                                    np.array([np.frombuffer(s.signature, np.uint8) for s in pc.signatures]),
                                    np.full(len(pc.signatures), 64, np.uint32))
            for mode in (T.MODE_COMMIT, T.MODE_LIGHT, T.MODE_LIGHT_TRUSTING):
                reqs.append((mode, pv, "kc", pbid(bid), cm.height, packed, 1, 3))
                exp.append(oracle_result(mode, vs, "kc", bid, cm.height, cm, 1, 3))
        got = T.verify_commits(engine, reqs)
        pb = T.PreparedBatch(reqs)
        pb.run(engine)
        for g, g2, e in zip(got, pb.errors(), exp):
            assert same(g, e) and same(g2, e), (g, g2, e)
    finally:
        engine.keyset_free(ks)


def test_keyset_index_past_the_key_set_is_einval(engine):
    """A key-set index past the key set fails the whole seam call with TMED_EINVAL (checked while
    the candidates are staged), before anything runs on the device."""
    import numpy as np
    from oracle.fixtures import make_block_id, make_commit, make_valset, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("kx", i) for i in range(6)], [10] * 6)
    bid = make_block_id("kx")
    cm = make_commit(vs, seeds, "kx", 7, 0, bid)
    pv, pc = to_product(vs, cm)
    pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators])
    ks = engine.keyset_load(pubs)
    pv.keyset = ks
    pv.keyset_index = np.arange(len(pubs), dtype=np.uint32)
    pv.keyset_index[3] = len(pubs)  # one past the end
    try:
        with pytest.raises(T.TmedError):
            T.verify_commits(engine, [(T.MODE_COMMIT, pv, "kx", pbid(bid), cm.height, pc, 0, 0)])
        pv.keyset_index[3] = 3
        assert T.verify_commits(engine, [(T.MODE_COMMIT, pv, "kx", pbid(bid), cm.height, pc, 0, 0)]) == [None]
    finally:
        engine.keyset_free(ks)


@pytest.mark.parametrize("batch,chain", [(1, "bs-chain"), (3, "bs-chain"), (256, "bs-chain"), (3, "c" * 200)])
@pytest.mark.parametrize("keyed", [False, True])
def test_blocksync_window_matches_light_loops(engine, batch, chain, keyed):
    """tmed_blocksync_verify (f4: pipelined LIGHT batches over one validator set) gives the
    reference VerifyCommitLight outcome for every block: valid commits, a bad signature
    before and after the 2/3 crossing, wrong height, wrong BlockID, not enough power; a
    200-character chain ID takes the pipeline's synchronous host-assembled fallback."""
    import numpy as np
    from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("bs", i) for i in range(7)], [10] * 7)
    blocks, exp, bids, heights = [], [], [], []
    for h in range(11):
        bid = make_block_id("bs%d" % h)
        cm = make_commit(vs, seeds, chain, 50 + h, 0, bid)
        want_h, want_bid = 50 + h, bid
        if h == 2:
            resign(cm, 0, seeds[0], "bad")          # before the crossing -> wrong signature (#0)
        elif h == 3:
            resign(cm, 6, seeds[6], "bad")          # after the crossing -> never verified, OK
        elif h == 4:
            want_h = 49                             # wrong height
        elif h == 5:
            want_bid = make_block_id("other")       # wrong block ID
        elif h == 6:
            for i in range(3, 7):                   # absent -> not enough power
                cm.signatures[i].flag = 1
                cm.signatures[i].signature = b""
        exp.append(oracle_result(T.MODE_LIGHT, vs, chain, want_bid, want_h, cm, 0, 0))
        _, pc = to_product(vs, cm)
        blocks.append(pc)
        bids.append(pbid(want_bid))
        heights.append(want_h)
    pv = to_product(vs, make_commit(vs, seeds, chain, 1, 0, make_block_id("x")))[0]
    ks = 0
    if keyed:
        ks = engine.keyset_load(np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators]))
        pv.keyset = ks
    try:
        w = T.BlocksyncWindow(pv, chain, bids, heights, blocks)
        w.run(engine, batch)
        for h, (g, e) in enumerate(zip(w.errors(), exp)):
            assert same(g, e), (h, g, e)
        ref = T.verify_commits(engine, [(T.MODE_LIGHT, pv, chain, b, hh, c, 0, 0)
                                        for b, hh, c in zip(bids, heights, blocks)])
        assert all(same(a, b) for a, b in zip(ref, w.errors()))
    finally:
        if ks:
            engine.keyset_free(ks)


def test_edge_scenarios_gpu(engine):
    """Unknown BlockIDFlags, malformed BlockID hashes and odd-length ValidatorAddresses (0/19/21
    bytes, and the 19-byte prefix of an address ending in 0x00) through the GPU seam: panics are
    reported per request at the reference loop's index (TMED_COMMIT_PANIC), GetByAddress matches by
    bytes.Equal, every other outcome equals the reference loops."""
    from commit_cases import edge_scenarios, oracle_outcome, same_outcome
    reqs, exp = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in edge_scenarios(seed=8, count=60):
        exp.append(oracle_outcome(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    got = T.verify_commits(engine, reqs)
    bad = [(q, got[q], exp[q]) for q in range(len(reqs)) if not same_outcome(got[q], exp[q])]
    assert not bad, bad[:5]
    assert any(isinstance(e, tuple) for e in exp)


@pytest.mark.parametrize("pinned", ["all", "alternate", "separate"])
@pytest.mark.parametrize("keyed", [False, True])
def test_blocksync_pinned_signatures_gpu(engine, pinned, keyed):
    """Signatures in tmed_host_alloc memory are DMA'd straight from the caller's arrays (batches of
    >= 1 MB staged): every block's outcome (code, index, signatures verified) equals the run from
    pageable memory — all commits pinned, every other commit pinned (mixed runs: staged and
    direct signatures in one batch), and one pinned allocation per commit (equal-length runs in
    different allocations are not merged into one 2-D copy: keyset.hip votes_enqueue) — with
    known-answer bad signatures before and after the 2/3 crossing and a short (63-byte) signature
    in a pinned run."""
    import hashlib
    import numpy as np
    from tmed import PinnedBuffer
    from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits
    nvals, nblk = 2000, 30  # 12-block batches of ~16k candidates: 1.4 MB staged, the copy-stream path
    seeds = seeds_from_tag(b"tmed-pin-key", 0, nvals)
    vals, order = make_valset(pubkeys_of(engine, seeds), [10] * nvals)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    upto = nvals * 2 // 3 + 1
    bids = [T.BlockID(hashlib.sha256(b"pin%d" % b).digest(), 7, hashlib.sha256(b"psh%d" % b).digest())
            for b in range(nblk)]
    specs = [(seeds[order], addrs, 100 + b, 0, bids[b], 1672531200 + b, None) for b in range(nblk)]

    def window(pin):
        commits = sign_commits(engine, "pin-chain", specs, sign_upto=upto)
        for b, c in enumerate(commits):
            if b % 5 == 1:
                c.sigs[(b * 31) % upto, 3] ^= 0x40      # before the crossing: wrong signature
            if b % 5 == 2:
                c.sigs[upto + 1, 9] ^= 0x01             # after it: never reached
            if b % 7 == 3:
                c.sig_lens[(b * 13) % upto] = 63        # a short signature: wrong length
        buf = []
        if pin and pinned == "separate":
            for c in commits:
                buf.append(PinnedBuffer(nvals * 64))
                a = buf[-1].array((nvals, 64), np.uint8)
                a[:] = c.sigs
                c.sigs = a
        elif pin:
            buf.append(PinnedBuffer(nblk * nvals * 64))
            a = buf[0].array((nblk * nvals, 64), np.uint8)
            for b, c in enumerate(commits):
                if pinned == "all" or b % 2 == 0:
                    a[b * nvals:(b + 1) * nvals] = c.sigs
                    c.sigs = a[b * nvals:(b + 1) * nvals]
        return T.BlocksyncWindow(vals, "pin-chain", bids, [100 + b for b in range(nblk)], commits), buf

    ks = 0
    if keyed:
        ks = engine.keyset_load(np.array([np.frombuffer(v.pub_key, np.uint8) for v in vals.validators]))
        vals.keyset = ks
    try:
        w0, _ = window(False)
        w0.run(engine, 12)
        w1, buf = window(True)
        w1.run(engine, 12)
        assert (w0.codes() == w1.codes()).all()
        assert (w0.verified() == w1.verified()).all()
        assert [w0.res[h].idx for h in range(nblk)] == [w1.res[h].idx for h in range(nblk)]
        assert (w0.codes() == 4).sum() >= 6 and (w0.codes() == 0).sum() >= 10
        for b in buf:
            b.free()
    finally:
        if ks:
            engine.keyset_free(ks)
            vals.keyset = 0


@pytest.mark.parametrize("keyed", [False, True])
def test_blocksync_stream_of_windows_gpu(engine, keyed):
    """tmed_blocksync_submit / tmed_blocksync_wait: windows submitted back to back (batches of one
    window still in flight when the next is queued, windows of 1, 5 and 12 blocks, pinned and
    pageable signatures) give exactly the per-window tmed_blocksync_verify results; every earlier
    window is final when submit returns; a tmed_verify_commits call between submits first collects
    the stream; the structs passed to submit may be rebuilt right after it returns."""
    import hashlib
    import numpy as np
    from tmed import PinnedBuffer
    from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits
    nvals = 1500
    seeds = seeds_from_tag(b"tmed-stream-key", 0, nvals)
    vals, order = make_valset(pubkeys_of(engine, seeds), [10] * nvals)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    upto = nvals * 2 // 3 + 1
    sizes = [12, 1, 5, 12, 7]
    bufs = []

    def window(k, b0, n, pin):
        bids = [T.BlockID(hashlib.sha256(b"st%d" % b).digest(), 3, hashlib.sha256(b"sp%d" % b).digest())
                for b in range(b0, b0 + n)]
        specs = [(seeds[order], addrs, 500 + b, 0, bids[b - b0], 1672531200 + b, None) for b in range(b0, b0 + n)]
        commits = sign_commits(engine, "stream-chain", specs, sign_upto=upto)
        for b, c in zip(range(b0, b0 + n), commits):
            if b % 4 == 1:
                c.sigs[(b * 37) % upto, 5] ^= 0x20      # before the crossing: wrong signature
            if b % 6 == 2:
                c.sigs[upto + 3, 1] ^= 0x02             # after it: never reached
        if pin:
            buf = PinnedBuffer(n * nvals * 64)
            a = buf.array((n * nvals, 64), np.uint8)
            for j, c in enumerate(commits):
                a[j * nvals:(j + 1) * nvals] = c.sigs
                c.sigs = a[j * nvals:(j + 1) * nvals]
            bufs.append(buf)
        return T.BlocksyncWindow(vals, "stream-chain", bids, [500 + b for b in range(b0, b0 + n)], commits)

    ks = 0
    if keyed:
        ks = engine.keyset_load(np.array([np.frombuffer(v.pub_key, np.uint8) for v in vals.validators]))
        vals.keyset = ks
    try:
        wins, b0 = [], 0
        for k, n in enumerate(sizes):
            wins.append(window(k, b0, n, pin=k % 2 == 0))
            b0 += n
        ref = []
        for w in wins:  # a call per window
            w.run(engine, 2)
            ref.append((w.codes().copy(), w.verified().copy(), [w.res[h].idx for h in range(w.n)]))
            w.res = type(w.res)()
        for k, w in enumerate(wins):
            w.submit(engine, 2)
            if k:  # the previous window is final now
                p = wins[k - 1]
                assert (p.codes() == ref[k - 1][0]).all() and (p.verified() == ref[k - 1][1]).all()
            if k == 2:  # another seam call collects the stream first
                c = wins[0].commits[0]
                got = T.verify_commits(engine, [(T.MODE_LIGHT, vals, "stream-chain", c.block_id, c.height, c, 0, 0)])
                assert got == [None]
            w.win = w.bids = w.ccs = w.vs = None  # the structs may go once submit returned
            if k == 3:  # a malformed window is refused without touching the windows in flight
                bad = window(9, 1000, 2, pin=False)
                bad.ccs[1].sigs = None  # a commit without its signature array: TMED_EINVAL
                with pytest.raises(T.TmedError):
                    bad.submit(engine, 2)
        T.blocksync_wait(engine)
        for w, (codes, vers, idx) in zip(wins, ref):
            assert (w.codes() == codes).all() and (w.verified() == vers).all()
            assert [w.res[h].idx for h in range(w.n)] == idx
        assert sum(int((r[0] == 4).sum()) for r in ref) >= 8
        T.blocksync_wait(engine)  # nothing in flight: a no-op
    finally:
        for b in bufs:
            b.free()
        if ks:
            engine.keyset_free(ks)
            vals.keyset = 0
