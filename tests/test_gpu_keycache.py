"""The commit seam's key-set cache on the GPU (csrc/keycache.h, keycache.hip; include/tmed25519.h
tmed_keycache_*): the reference's callers pass validator sets WITHOUT key-set handles, as the
drop-in patch of INTEGRATION.md does, and must reach the key-cached kernels after the first call,
with decisions, error values and Got/Needed equal to the oracle's restatement of the reference
loops (types/validator_set.go:667-826) on every call — cold, warm, after a pool reset, with a wrong
set_hash.  Shapes: C1 (state/validation.go:93-96: LastCommit against LastValidators every block),
C3 (light/verifier.go:58,73-76: per-height sets changing by one key), a blocksync window
(blockchain/v0/reactor.go:366-367).  tmed_keyset_extend (pooled explicit key sets) is checked too."""
import numpy as np
import pytest

from conftest import engine_with_env
from oracle import commit as C
import tmed.types as T
from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits
from test_gpu_configs import CHAIN, T2023, _bid, _copy, _corrupt, _ocommit, _oracle, _ovals, _port_verify, _same

pytestmark = pytest.mark.gpu


@pytest.fixture
def cached():
    """A fresh context with the key-set cache on (the product default) and an 8 GiB pool budget."""
    e = engine_with_env(TMED_KEYCACHE=1)
    e.keycache_config(True, 8 << 30)
    yield e
    e.close()


_PER_KEY = 33 + 32 * 129 * 128 + (20 * 2049 + 4225) * 128  # keyset_bytes_per_key with the radix-2^12 comb


def _delta(a, b):
    return {k: b[k] - a[k] for k in ("lookups", "hits", "keyed_sets", "generic_sets", "keys_appended",
                                     "keys_deferred", "pool_resets", "keyed_sigs", "generic_sigs")}


def _c1(eng, tag=b"tmed-bench-key", n=175):
    seeds = seeds_from_tag(tag, 0, n)
    pubs = pubkeys_of(eng, seeds)
    vals, order = make_valset(pubs, [10] * n)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    bid = _bid(b"kc-" + tag)
    base = sign_commits(eng, CHAIN, [(seeds[order], addrs, 3, 0, bid, T2023, None)])[0]
    return vals, bid, base


def _c1_requests(vals, bid, base):
    ovs = _ovals(vals)
    reqs, exp = [], []
    for bad in (None, 0, 174, 116, 150):
        pc = _copy(base)
        if bad is not None:
            _corrupt(pc, bad)
        oc = _ocommit(pc)
        for req in ((T.MODE_COMMIT, vals, CHAIN, bid, 3, pc, 0, 0), (T.MODE_LIGHT, vals, CHAIN, bid, 3, pc, 0, 0),
                    (T.MODE_LIGHT_TRUSTING, vals, CHAIN, None, 0, pc, 1, 3)):
            reqs.append(req)
            exp.append(_oracle(req, ovs, oc))
    return reqs, exp


def test_c1_first_call_generic_then_keyed(cached):
    """The first VerifyCommit against a new set runs the generic kernels and queues its keys; every
    later call is keyed (the first by a pooled-key miss, the rest cache hits) — decisions equal the
    oracle loops on every call, bad signatures at 0 / 116 / 150 / 174 included."""
    vals, bid, base = _c1(cached)
    reqs, exp = _c1_requests(vals, bid, base)
    s0 = cached.keycache_stats()
    first = T.verify_commits(cached, [reqs[0]])[0]
    cached.keycache_wait()  # the context's worker builds the queued keys after the call
    d = _delta(s0, cached.keycache_stats())
    assert _same(first, exp[0])
    assert d["generic_sets"] == 1 and d["keyed_sets"] == 0 and d["keys_deferred"] == 175
    s1 = cached.keycache_stats()
    assert s1["pool_keys"] == 175 and s1["pending_keys"] == 0
    got = [T.verify_commits(cached, [r])[0] for r in reqs]
    d = _delta(s1, cached.keycache_stats())
    assert d["keyed_sets"] == len(reqs) and d["generic_sets"] == 0 and d["hits"] == len(reqs) - 1
    assert d["keys_appended"] == 0
    for q in range(len(reqs)):
        assert _same(got[q], exp[q]), (q, got[q], exp[q])
    batch = T.verify_commits(cached, reqs)  # the same requests as one batch: one cached set
    for q in range(len(reqs)):
        assert _same(batch[q], exp[q]), (q, batch[q], exp[q])
    # the cache off: the generic kernels again, same answers
    cached.keycache_config(False)
    s2 = cached.keycache_stats()
    off = T.verify_commits(cached, reqs)
    assert cached.keycache_stats()["lookups"] == s2["lookups"]
    for q in range(len(reqs)):
        assert _same(off[q], exp[q]), (q, off[q], exp[q])


def test_c3_changing_sets_without_handles(cached):
    """C3 shape through the cache: 40 headers x 175 validators, the set changing one key per height,
    per header Trusting(1/3) against set h and Light against set h + 2, header 5 against a set 120
    heights back (Got 530 <= Needed 583), bad signatures in headers 9 and 17 (inside the Trusting
    prefix) and 23 (after the Light crossing).  Call 1 is cold (generic, keys queued), call 2 is
    keyed with every key built once in the shared pool, call 3 hits; a sliding call adds one new set
    per height.  Every call equals the oracle loops."""
    nv, H, gap, far = 175, 40, 2, 120
    pool_seeds = seeds_from_tag(b"tmed-c3-key", 0, H + gap + nv + far + 4)
    pool_pubs = pubkeys_of(cached, pool_seeds)
    sets, specs = {}, []
    hs = sorted(set(range(H + gap + 4)) | {far + 5 + gap})
    for h in hs:
        vals, order = make_valset(pool_pubs[h:h + nv], [10] * nv)
        sets[h] = vals
        addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
        specs.append((pool_seeds[h:h + nv][order], addrs, h + 1, 0, _bid(b"c3-%d" % (h + 1)), T2023 + h, None))
    commits = dict(zip(hs, sign_commits(cached, CHAIN, specs)))
    _corrupt(commits[9 + gap], 3)
    _corrupt(commits[17 + gap], 40)
    _corrupt(commits[23 + gap], 160)
    osets = {h: _ovals(v) for h, v in sets.items()}

    def batch(lo, hi):
        reqs, exp = [], []
        for h in range(lo, hi):
            u = h + gap if h != 5 else far + 5 + gap
            pc = commits[u]
            oc = _ocommit(pc)
            for req, ovs in (((T.MODE_LIGHT_TRUSTING, sets[h], CHAIN, None, 0, pc, 1, 3), osets[h]),
                             ((T.MODE_LIGHT, sets[u], CHAIN, pc.block_id, u + 1, pc, 0, 0), osets[u])):
                reqs.append(req)
                exp.append(_oracle(req, ovs, oc))
        return reqs, exp

    reqs, exp = batch(0, H)
    used = set(range(H)) | {h + gap for h in range(H) if h != 5} | {far + 5 + gap}
    distinct = {pool_pubs[i].tobytes() for h in used for i in range(h, h + nv)}
    for call in range(3):
        s0 = cached.keycache_stats()
        got = T.verify_commits(cached, reqs)
        cached.keycache_wait()
        d = _delta(s0, cached.keycache_stats())
        bad = [(q, str(got[q]), str(exp[q])) for q in range(len(reqs)) if not _same(got[q], exp[q])]
        assert not bad, (call, bad[:4])
        if call == 0:
            assert d["keyed_sets"] == 0 and d["keys_deferred"] > 0
        else:
            assert d["generic_sets"] == 0 and d["keyed_sigs"] > 0 and d["keys_appended"] == 0
        if call == 2:
            assert d["hits"] == d["lookups"]
    assert isinstance(exp[10], C.ErrNotEnoughVotingPowerSigned)
    assert (exp[10].got, exp[10].needed) == (10 * (nv - far - gap), 583)
    assert cached.keycache_stats()["pool_keys"] == len(distinct)  # each key built once
    # slide by two heights: two new sets, whose keys the pool already holds (the far set 127 covers
    # keys 127..301): keyed at once by pooled-key misses, the rest are hits, nothing is built
    reqs2, exp2 = batch(2, H + 2)
    s0 = cached.keycache_stats()
    got = T.verify_commits(cached, reqs2)
    d = _delta(s0, cached.keycache_stats())
    assert all(_same(got[q], exp2[q]) for q in range(len(reqs2)))
    assert d["keyed_sets"] == d["lookups"] and d["hits"] == d["lookups"] - 2 and d["keys_appended"] == 0


def test_blocksync_window_builds_its_keys_first(cached, engine):
    """A blocksync window whose signatures pay for its keys (64 validators x 4,096 blocks: 43
    signatures per block, 176k >= 2048 x 64) is keyed on its FIRST call; a small window of a new set
    is generic once.  Outcomes equal the cache-off generic path on every block and the oracle on
    the corrupted ones (bad signature before the crossing -> wrong signature; after it -> ok)."""
    nv, nb = 64, 4096
    seeds = seeds_from_tag(b"tmed-kc-bs", 0, nv)
    pubs = pubkeys_of(cached, seeds)
    vals, order = make_valset(pubs, [10] * nv)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    upto = nv * 2 // 3 + 1
    specs = [(seeds[order], addrs, b + 1, 0, _bid(b"kcbs-%d" % b), T2023 + b, None) for b in range(nb)]
    commits = sign_commits(cached, CHAIN, specs, sign_upto=upto)
    for b in range(3, nb, 97):
        _corrupt(commits[b], (b * 31) % upto)
    for b in range(50, nb, 101):
        _corrupt(commits[b], upto)  # past the crossing: never reached
    bids = [c.block_id for c in commits]
    heights = [c.height for c in commits]
    s0 = cached.keycache_stats()
    win = T.BlocksyncWindow(vals, CHAIN, bids, heights, commits)
    win.run(cached, 128)
    d = _delta(s0, cached.keycache_stats())
    assert d["keyed_sets"] == 1 and d["generic_sets"] == 0 and d["keys_appended"] == nv and d["keys_deferred"] == 0
    ref = T.BlocksyncWindow(vals, CHAIN, bids, heights, commits)
    ref.run(engine, 128)  # cache off: generic kernels
    assert (win.codes() == ref.codes()).all() and (win.verified() == ref.verified()).all()
    ovs = _ovals(vals)
    for b in list(range(3, nb, 97))[:6] + list(range(50, nb, 101))[:4] + [0, 1]:
        e = C.verify_commit_light(ovs, CHAIN, C.BlockID(bids[b].hash, bids[b].psh_total, bids[b].psh_hash),
                                  heights[b], _ocommit(commits[b]), _port_verify)
        assert _same(win.errors()[b], e), (b, win.errors()[b], e)
    # a small window against a NEW set: generic now, keyed next time
    vals2, order2 = make_valset(pubkeys_of(cached, seeds_from_tag(b"tmed-kc-bs2", 0, nv)), [10] * nv)
    w2 = T.BlocksyncWindow(vals2, CHAIN, bids[:2], heights[:2], commits[:2])  # signed by other keys: fails
    s0 = cached.keycache_stats()
    w2.run(cached, 0)
    cached.keycache_wait()
    assert _delta(s0, cached.keycache_stats())["generic_sets"] == 1
    w2.run(cached, 0)
    assert _delta(s0, cached.keycache_stats())["keyed_sets"] == 1
    assert all(str(e).startswith("wrong signature (#0)") for e in w2.errors())


def test_budget_resets_and_wrong_set_hash(cached):
    """A pool budget of ~300 keys: two 175-key sets alternately warmed reset the pool each time;
    one set_hash given for two different sets (a stale / wrong hash) is caught by the key compare.
    Every call equals the oracle."""
    a = _c1(cached, b"kc-A")
    b = _c1(cached, b"kc-B")
    cached.keycache_config(True, 300 * _PER_KEY)
    ra, ea = _c1_requests(*a)
    rb, eb = _c1_requests(*b)
    for rnd in range(2):
        for (reqs, exp, vals) in ((ra, ea, a[0]), (rb, eb, b[0])):
            cached.keycache_warm(vals)  # builds its keys now (resetting the pool for the other set)
            s0 = cached.keycache_stats()
            got = T.verify_commits(cached, reqs)
            assert _delta(s0, cached.keycache_stats())["keyed_sets"] == 1
            bad = [(q, str(got[q]), str(exp[q])) for q in range(len(reqs)) if not _same(got[q], exp[q])]
            assert not bad, (rnd, bad[:3], cached.keycache_stats())
    assert cached.keycache_stats()["pool_resets"] >= 3
    cached.keycache_config(True, 8 << 30)
    h = bytes(range(32))
    a[0].set_hash = h
    b[0].set_hash = h
    try:
        for _ in range(2):
            for (reqs, exp) in ((ra, ea), (rb, eb)):
                got = T.verify_commits(cached, reqs)
                cached.keycache_wait()
                bad = [(q, str(got[q]), str(exp[q])) for q in range(len(reqs)) if not _same(got[q], exp[q])]
                assert not bad, (bad[:3], cached.keycache_stats())
    finally:
        a[0].set_hash = b[0].set_hash = None


def test_keyset_extend_keeps_indexes(cached):
    """tmed_keyset_extend: a 100-key set extended by 75 keys; a 175-validator commit verified by
    keyset_index into the extended set (keys of both halves) equals the oracle; old indexes stay."""
    vals, bid, base = _c1(cached, b"kc-ext")
    pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in vals.validators])
    ks = cached.keyset_load(pubs[75:])                    # validators 75..174 at indexes 0..99
    try:
        assert cached.keyset_extend(ks, pubs[:75]) == 100  # validators 0..74 at 100..174
        assert cached.keyset_extend(ks, pubs[:0]) == 175
        v2 = T.ValidatorSet(list(vals.validators))
        v2.keyset = ks
        v2.keyset_index = np.concatenate([np.arange(100, 175), np.arange(0, 100)]).astype(np.uint32)
        reqs, exp = _c1_requests(v2, bid, base)
        got = T.verify_commits(cached, reqs)
        assert all(_same(got[q], exp[q]) for q in range(len(reqs)))
        s = cached.keycache_stats()
        assert s["lookups"] == 0  # a set with a handle never reaches the cache
    finally:
        cached.keyset_free(ks)


def _bs_window(eng, tag, nv=64, nb=4096):
    """A blocksync window (default 64 validators x 4,096 blocks, VerifyCommitLight per block) whose
    signatures pay for its keys: keyed, through the throughput kernels, on its first call."""
    seeds = seeds_from_tag(tag, 0, nv)
    vals, order = make_valset(pubkeys_of(eng, seeds), [10] * nv)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    upto = nv * 2 // 3 + 1
    specs = [(seeds[order], addrs, b + 1, 0, _bid(tag + b"-%d" % b), T2023 + b, None) for b in range(nb)]
    commits = sign_commits(eng, CHAIN, specs, sign_upto=upto)
    for b in range(5, nb, 89):
        _corrupt(commits[b], (b * 7) % upto)
    return vals, CHAIN, [c.block_id for c in commits], [c.height for c in commits], commits


def test_pool_grows_under_throughput_batches(engine):
    """The pool grows while its radix-2^12 combs are in use: window A's 64 keys are built (combs of
    both radixes, throughput kernels), then window B's 64 keys are appended (the pool's chunk gains
    keys, the radix-2^12 comb is extended for them), then A runs again over the keys built before.
    Every outcome equals the cache-off generic path's."""
    eng = engine_with_env(TMED_KEYCACHE=1)
    try:
        eng.keycache_config(True, 8 << 30)
        wins = [_bs_window(eng, t) for t in (b"kc-grow-A", b"kc-grow-B")]
        refs = []
        for w in wins:
            r = T.BlocksyncWindow(*w)
            r.run(engine, 128)
            refs.append(r)
        for i in (0, 1, 0, 1):
            s0 = eng.keycache_stats()
            got = T.BlocksyncWindow(*wins[i])
            got.run(eng, 128)
            d = _delta(s0, eng.keycache_stats())
            assert d["keyed_sets"] == 1 and d["generic_sets"] == 0
            assert (got.codes() == refs[i].codes()).all() and (got.verified() == refs[i].verified()).all(), i
            assert not got.codes().all() and got.codes().any()  # both outcomes present
        assert eng.keycache_stats()["pool_keys"] == 128
        # the budget shrinks below the pool: the pool is dropped at once (its memory freed, not
        # kept for reuse) and A's next call builds its keys again, in plain allocations
        eng.keycache_config(True, 64 * _PER_KEY)
        assert eng.keycache_stats()["pool_keys"] == 0
        s0 = eng.keycache_stats()
        got = T.BlocksyncWindow(*wins[0])
        got.run(eng, 128)
        assert (got.codes() == refs[0].codes()).all() and (got.verified() == refs[0].verified()).all()
        assert _delta(s0, eng.keycache_stats())["keys_appended"] == 64 and eng.keycache_stats()["pool_keys"] == 64
    finally:
        eng.close()


def test_pool_partial_chunk_replaced_after_budget_grows(engine):
    """The pool's comb chunks (512 keys each) are whole up to its budget, so a budget of 700 keys
    leaves chunk 1 holding 188.  A set of 600 validators is warmed and verified through the
    throughput kernels (both combs built, chunk 1 partial); the budget then grows to 2,000 keys and
    a set of 300 new validators is warmed: chunk 1 is replaced by a whole one with its 88 built keys
    copied over (radix-256 comb at the append, radix-2^12 comb at the next throughput batch).  Both
    sets' windows, before and after, equal the cache-off generic path's."""
    eng = engine_with_env(TMED_KEYCACHE=1)
    try:
        eng.keycache_config(True, 700 * _PER_KEY)
        wa = _bs_window(eng, b"kc-part-A", nv=600, nb=64)
        wb = _bs_window(eng, b"kc-part-B", nv=300, nb=96)
        refs = []
        for w in (wa, wb):
            r = T.BlocksyncWindow(*w)
            r.run(engine, 64)
            refs.append(r)

        def run(i, w):
            s0 = eng.keycache_stats()
            got = T.BlocksyncWindow(*w)
            got.run(eng, 64)
            assert _delta(s0, eng.keycache_stats())["keyed_sets"] == 1
            assert (got.codes() == refs[i].codes()).all() and (got.verified() == refs[i].verified()).all(), i

        eng.keycache_warm(wa[0])
        assert eng.keycache_stats()["pool_keys"] == 600
        run(0, wa)
        eng.keycache_config(True, 2000 * _PER_KEY)
        eng.keycache_warm(wb[0])
        assert eng.keycache_stats()["pool_keys"] == 900
        run(1, wb)
        run(0, wa)
    finally:
        eng.close()
