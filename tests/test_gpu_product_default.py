"""The drop-in's PRODUCT DEFAULT on the GPU: the key-set cache on (tmed_init's default, what the
Go shim and INTEGRATION.md's patch get), validator sets passed WITHOUT key-set handles.  The rest
of the commit suite runs on the shared cache-off `engine` so that each test exercises the kernel
path it names; this file runs the same parity corpus, the concurrency pattern of the reference's
callers and the context teardown on cache-on contexts, against the oracle's restatement of the
reference loops (types/validator_set.go:667-826; light/verifier.go:58-76) with the C port as the
per-signature verifier.  Counters (tmed_keycache_stats) show which calls were keyed."""
import hashlib
import threading

import numpy as np
import pytest

from commit_cases import edge_scenarios, oracle_outcome, pbid, same_outcome, scenarios
from conftest import engine_with_env
from oracle import commit as C
import tmed.types as T
from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits
from test_gpu_configs import CHAIN, T2023, _bid, _copy, _corrupt, _ocommit, _oracle, _ovals, _port_verify, _same

pytestmark = pytest.mark.gpu


def _cache_on():
    e = engine_with_env(TMED_KEYCACHE=1)
    e.keycache_config(True, 16 << 30)
    return e


@pytest.fixture
def product():
    """A fresh cache-on context per test (a cold pool: the first call of every set is generic)."""
    e = _cache_on()
    yield e
    e.close()


def _delta(a, b):
    return {k: b[k] - a[k] for k in ("lookups", "hits", "keyed_sets", "generic_sets", "keys_appended",
                                     "keys_deferred", "pool_resets", "keyed_sigs", "generic_sigs")}


def _corpus(seed, edge_seed):
    reqs, exp = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=seed, count=120):
        exp.append(oracle_outcome(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in edge_scenarios(seed=edge_seed, count=60):
        exp.append(oracle_outcome(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    return reqs, exp


@pytest.mark.parametrize("pipe", [None, "64"])
def test_commit_corpus_cache_on(product, monkeypatch, pipe):
    """The seam's random corpus (bad / short / other-chain signatures, double votes, Trusting sets
    that differ from the commit's, duplicate addresses) and its edge corpus (unknown BlockIDFlags,
    malformed BlockID hashes: Go's panics at the loop's index; 0/19/21-byte addresses) through a
    cache-on context: call 1 cold (generic, every set's keys deferred to the context's worker),
    call 2 with every set keyed from the pool, then every seventh request alone (the key-cached
    latency kernels).  pipe: TMED_PIPE_SIGS=64, many tiny batches through the pipelined seam."""
    reqs, exp = _corpus(2 if pipe is None else 3, 8 if pipe is None else 9)
    if pipe:
        monkeypatch.setenv("TMED_PIPE_SIGS", pipe)
    s0 = product.keycache_stats()
    got1 = T.verify_commits(product, reqs)
    product.keycache_wait()
    s1 = product.keycache_stats()
    d1 = _delta(s0, s1)
    assert d1["keyed_sets"] == 0 and d1["generic_sets"] > 0 and d1["keys_deferred"] > 0, d1
    got2 = T.verify_commits(product, reqs)
    d2 = _delta(s1, product.keycache_stats())
    assert d2["generic_sets"] == 0 and d2["keyed_sets"] == d2["lookups"] > 0 and d2["keys_appended"] == 0, d2
    for call, got in (("cold", got1), ("keyed", got2)):
        bad = [(q, got[q], exp[q]) for q in range(len(reqs)) if not same_outcome(got[q], exp[q])]
        assert not bad, (call, bad[:5])
    for q in range(0, len(reqs), 7):
        one = T.verify_commits(product, [reqs[q]])[0]
        assert same_outcome(one, exp[q]), (q, one, exp[q])
    assert any(isinstance(e, tuple) for e in exp) and sum(e is not None for e in exp) > 20


@pytest.mark.parametrize("pinned", [False, True])
def test_blocksync_stream_cache_on(product, pinned):
    """A replay as the drop-in runs it: windows of one set (without a handle) submitted back to back
    through tmed_blocksync_submit.  The first windows' signatures do not pay for the set's keys
    (6 blocks x 1,200 validators < 2,048 per key): windows 0 and 1 run generic; submitting window 1
    collects window 0, whose release wakes the context's worker, which builds the keys while
    window 1 is still in flight; windows 2-5 are keyed and alternate between the two kernel lanes.
    Every block equals the oracle's VerifyCommitLight, bad signatures before and after the 2/3
    crossing included."""
    from tmed import PinnedBuffer
    nv, nwin, per = 1200, 6, 6
    seeds = seeds_from_tag(b"tmed-pd-bs%d" % pinned, 0, nv)
    vals, order = make_valset(pubkeys_of(product, seeds), [10] * nv)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    upto = nv * 2 // 3 + 1
    nb = nwin * per
    bids = [T.BlockID(hashlib.sha256(b"pdbs%d" % b).digest(), 5, hashlib.sha256(b"pdps%d" % b).digest())
            for b in range(nb)]
    specs = [(seeds[order], addrs, 700 + b, 0, bids[b], T2023 + b, None) for b in range(nb)]
    commits = sign_commits(product, "pd-chain", specs, sign_upto=upto)
    for b, c in enumerate(commits):
        if b % 5 == 1:
            _corrupt(c, (b * 37) % upto)   # before the crossing: wrong signature
        if b % 7 == 2:
            _corrupt(c, upto + 2)          # after it: never reached
    bufs = []
    if pinned:
        buf = PinnedBuffer(nb * nv * 64)
        a = buf.array((nb * nv, 64), np.uint8)
        for b, c in enumerate(commits):
            a[b * nv:(b + 1) * nv] = c.sigs
            c.sigs = a[b * nv:(b + 1) * nv]
        bufs.append(buf)
    ovs = _ovals(vals)
    exp = [C.verify_commit_light(ovs, "pd-chain", C.BlockID(bids[b].hash, bids[b].psh_total, bids[b].psh_hash),
                                 700 + b, _ocommit(commits[b]), _port_verify) for b in range(nb)]
    try:
        wins = [T.BlocksyncWindow(vals, "pd-chain", bids[w * per:(w + 1) * per],
                                  [700 + b for b in range(w * per, (w + 1) * per)], commits[w * per:(w + 1) * per])
                for w in range(nwin)]
        s0 = product.keycache_stats()
        for k, w in enumerate(wins):
            w.submit(product, 2)
            if k == 1:
                product.keycache_wait()  # the worker (woken by window 0's release) has built the keys
        T.blocksync_wait(product)
        d = _delta(s0, product.keycache_stats())
        assert d["generic_sets"] == 2 and d["keyed_sets"] == nwin - 2 and d["keys_deferred"] == nv, d
        got = [e for w in wins for e in w.errors()]
        bad = [(b, str(got[b]), str(exp[b])) for b in range(nb) if not _same(got[b], exp[b])]
        assert not bad, bad[:4]
        assert sum(str(e).startswith("wrong signature") for e in exp) >= 6
    finally:
        for b in bufs:
            b.free()


def test_concurrent_callers_cache_on(product):
    """The reference's concurrent callers on ONE cache-on context (SURVEY §8b "Threading"): a
    blocksync replay submitting windows, a consensus-like caller running single VerifyCommits on a
    set that changes every three calls (so the worker's deferred key builds overlap the other
    callers' batches in flight), and a light client running Trusting + Light batches.  Every result
    equals the oracle loops."""
    # blocksync: 1,000 validators, windows of 4 blocks
    nv, nwin, per = 1000, 5, 4
    seeds = seeds_from_tag(b"tmed-pd-cc-bs", 0, nv)
    bvals, border = make_valset(pubkeys_of(product, seeds), [10] * nv)
    baddrs = np.array([np.frombuffer(v.address, np.uint8) for v in bvals.validators])
    upto = nv * 2 // 3 + 1
    nb = nwin * per
    bbids = [_bid(b"pdcc%d" % b) for b in range(nb)]
    bcommits = sign_commits(product, CHAIN, [(seeds[border], baddrs, 900 + b, 0, bbids[b], T2023 + b, None)
                                             for b in range(nb)], sign_upto=upto)
    for b in range(1, nb, 3):
        _corrupt(bcommits[b], (b * 53) % upto)
    bovs = _ovals(bvals)
    bexp = [C.verify_commit_light(bovs, CHAIN, C.BlockID(bbids[b].hash, bbids[b].psh_total, bbids[b].psh_hash),
                                  900 + b, _ocommit(bcommits[b]), _port_verify) for b in range(nb)]

    # consensus-like: 6 sets of 175 (each new), 3 single-commit calls per set, one bad signature in two
    c1 = []
    for k in range(6):
        s = seeds_from_tag(b"tmed-pd-cc-c1-%d" % k, 0, 175)
        vals, order = make_valset(pubkeys_of(product, s), [10] * 175)
        addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
        bid = _bid(b"pdc1-%d" % k)
        base = sign_commits(product, CHAIN, [(s[order], addrs, 3, 0, bid, T2023, None)])[0]
        ovs = _ovals(vals)
        for j in range(3):
            pc = _copy(base)
            if (k + j) % 2:
                _corrupt(pc, (k * 41 + j * 17) % 175)
            req = (T.MODE_COMMIT, vals, CHAIN, bid, 3, pc, 0, 0)
            c1.append((req, _oracle(req, ovs, _ocommit(pc))))

    # light client: 24 headers x 175, one key changing per height
    lnv, H, gap = 175, 24, 2
    lseeds = seeds_from_tag(b"tmed-pd-cc-lc", 0, H + gap + lnv)
    lpubs = pubkeys_of(product, lseeds)
    sets, specs = {}, []
    for h in range(H + gap):
        vals, order = make_valset(lpubs[h:h + lnv], [10] * lnv)
        sets[h] = vals
        addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
        specs.append((lseeds[h:h + lnv][order], addrs, h + 1, 0, _bid(b"pdlc-%d" % (h + 1)), T2023 + h, None))
    lcommits = dict(zip(range(H + gap), sign_commits(product, CHAIN, specs)))
    _corrupt(lcommits[4 + gap], 2)
    _corrupt(lcommits[13 + gap], 150)
    osets = {h: _ovals(v) for h, v in sets.items()}
    lreqs, lexp = [], []
    for h in range(H):
        pc = lcommits[h + gap]
        oc = _ocommit(pc)
        for req, ovs in (((T.MODE_LIGHT_TRUSTING, sets[h], CHAIN, None, 0, pc, 1, 3), osets[h]),
                         ((T.MODE_LIGHT, sets[h + gap], CHAIN, pc.block_id, h + gap + 1, pc, 0, 0), osets[h + gap])):
            lreqs.append(req)
            lexp.append(_oracle(req, ovs, oc))

    errors = []

    def run(name, fn, reps):
        try:
            for _ in range(reps):
                fn()
        except Exception as e:  # reported below with the failing caller's name
            errors.append("%s: %r" % (name, e))

    def blocksync():
        wins = [T.BlocksyncWindow(bvals, CHAIN, bbids[w * per:(w + 1) * per],
                                  [900 + b for b in range(w * per, (w + 1) * per)], bcommits[w * per:(w + 1) * per])
                for w in range(nwin)]
        for w in wins:
            w.submit(product, 2)
        T.blocksync_wait(product)
        got = [e for w in wins for e in w.errors()]
        bad = [b for b in range(nb) if not _same(got[b], bexp[b])]
        assert not bad, [(b, str(got[b]), str(bexp[b])) for b in bad[:3]]

    def consensus():
        for req, e in c1:
            g = T.verify_commits(product, [req])[0]
            assert _same(g, e), (str(g), str(e))

    def light():
        got = T.verify_commits(product, lreqs)
        bad = [q for q in range(len(lreqs)) if not _same(got[q], lexp[q])]
        assert not bad, [(q, str(got[q]), str(lexp[q])) for q in bad[:3]]

    s0 = product.keycache_stats()
    ths = [threading.Thread(target=run, args=j) for j in
           (("blocksync", blocksync, 3), ("consensus", consensus, 2), ("light", light, 4))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ths), "a caller did not finish"
    assert not errors, errors
    d = _delta(s0, product.keycache_stats())
    assert d["keys_deferred"] > 0, d
    product.keycache_wait()  # afterwards every set of the three callers is keyed
    s1 = product.keycache_stats()
    light()
    consensus()
    d = _delta(s1, product.keycache_stats())
    assert d["generic_sets"] == 0 and d["keyed_sets"] == d["lookups"] > 0, d
    assert sum(e is not None for _, e in c1) >= 6 and sum(e is not None for e in lexp) >= 2


def test_close_while_the_worker_builds_keys():
    """tmed_destroy right after a generic call that queued keys (no tmed_keycache_wait), and right
    after submitting a window that is still in flight: the context's key-build worker is joined
    before any staging buffer, event or stream it uses is freed (a use-after-free before round 5).
    The call's own result is final and equals the oracle."""
    for k in range(3):
        e = _cache_on()
        try:
            s = seeds_from_tag(b"tmed-pd-close-%d" % k, 0, 175)
            vals, order = make_valset(pubkeys_of(e, s), [10] * 175)
            addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
            bid = _bid(b"pdclose-%d" % k)
            pc = sign_commits(e, CHAIN, [(s[order], addrs, 3, 0, bid, T2023, None)])[0]
            _corrupt(pc, 3 * k + 1)
            req = (T.MODE_COMMIT, vals, CHAIN, bid, 3, pc, 0, 0)
            exp = _oracle(req, _ovals(vals), _ocommit(pc))
            got = T.verify_commits(e, [req])[0]
            assert _same(got, exp), (str(got), str(exp))
            if k == 2:  # a window in flight at close
                w = T.BlocksyncWindow(vals, CHAIN, [bid] * 8, [3] * 8, [pc] * 8)
                w.submit(e, 2)
        finally:
            e.close()
