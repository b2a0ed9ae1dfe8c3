"""The commit seam's key-set cache policy (tendermint-fork_amd/csrc/keycache.h) on the CPU.

tests/native/keycache_test.cpp builds the same header over a host stand-in for the device pool,
so every policy decision is checked without a GPU: a set seen for the first time by a small call
(C1: the first VerifyCommit after a set change) stays generic and its keys are built right after
the call; the next call is keyed, the one after is a cache hit; a call whose signatures pay for its
new keys builds them first; a light client's per-height sets share pooled keys; the HBM budget
resets the pool only when no other call holds indexes into it; a hit is always compared key by
key (a stale or wrong set_hash can only cost a miss); entries are bounded (LRU).  The cache key is
ValidatorSet.Hash() (types/validator_set.go:347-353) when the caller passes it.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AMORTIZE = 2048  # keycache.h kKcAmortizeSigsPerKey
FIELDS = ("lookups", "hits", "keyed_sets", "generic_sets", "keyed_sigs", "generic_sigs", "keys_appended",
          "keys_deferred", "pool_resets", "sets_evicted", "pool_keys", "sets_cached", "pending_keys", "backend_keys")


@pytest.fixture(scope="module")
def kct():
    d = os.path.join(ROOT, "tests", "native")
    subprocess.check_call(["make", "-s", "-C", d, "libkctest.so"])
    l = ctypes.CDLL(os.path.join(d, "libkctest.so"))
    P, SZ = ctypes.c_void_p, ctypes.c_size_t
    l.kct_new.restype = P
    l.kct_new.argtypes = [SZ]
    l.kct_free.argtypes = [P]
    l.kct_limits.argtypes = [P, SZ, SZ]
    l.kct_pin.argtypes = [P]
    l.kct_unpin.argtypes = [P]
    l.kct_fail_next_append.argtypes = [P]
    l.kct_lookup.restype = ctypes.c_int
    l.kct_lookup.argtypes = [P, P, SZ, P, SZ, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    l.kct_missing.restype = SZ
    l.kct_missing.argtypes = [P, P, SZ]
    l.kct_drain.restype = ctypes.c_int
    l.kct_drain.argtypes = [P]
    l.kct_stats.argtypes = [P, P]
    l.kct_pool_key.restype = ctypes.c_int
    l.kct_pool_key.argtypes = [P, ctypes.c_uint32, P]
    l.kct_digest.argtypes = [P, SZ, P]
    l.kct_retired.restype = SZ
    l.kct_retired.argtypes = [P]
    l.kct_all_pooled.restype = ctypes.c_int
    l.kct_all_pooled.argtypes = [P, P, SZ]
    l.kct_defer.argtypes = [P, P, SZ, SZ]
    return l


class Cache:
    def __init__(self, l, cap):
        self.l, self.h = l, l.kct_new(cap)

    def close(self):
        self.l.kct_free(self.h)

    def lookup(self, pubs, sigs, set_hash=None, may_reset=True, force=False, fast=True):
        pubs = np.ascontiguousarray(pubs, np.uint8)
        n = pubs.shape[0]
        idx = np.zeros(max(n, 1), np.uint32)
        hb = None if set_hash is None else ctypes.c_char_p(bytes(set_hash))
        k = self.l.kct_lookup(self.h, pubs.ctypes.data, n, hb, sigs, int(may_reset), int(force), int(fast),
                              idx.ctypes.data)
        return bool(k), idx[:n]

    def call(self, sets_sigs, **kw):
        """One seam call: pin, look every set up, unpin, drain (as commit.hip KcCall does)."""
        self.l.kct_pin(self.h)
        out = []
        any_keyed = False
        for pubs, sigs in sets_sigs:
            k, idx = self.lookup(pubs, sigs, may_reset=not any_keyed, **kw)
            any_keyed |= k
            out.append((k, idx))
        self.l.kct_unpin(self.h)
        assert self.l.kct_drain(self.h) == 0
        return out

    def stats(self):
        a = np.zeros(len(FIELDS), np.uint64)
        self.l.kct_stats(self.h, a.ctypes.data)
        return dict(zip(FIELDS, (int(x) for x in a)))

    def pool_key(self, i):
        b = ctypes.create_string_buffer(32)
        assert self.l.kct_pool_key(self.h, int(i), b) == 0
        return b.raw


def keys(tag, lo, hi):
    return np.array([np.frombuffer(hashlib.sha256(b"%s-%d" % (tag, i)).digest(), np.uint8) for i in range(lo, hi)])


def check_idx(c, pubs, idx):
    """every validator's pool index holds exactly its key"""
    for i in range(len(pubs)):
        assert c.pool_key(idx[i]) == pubs[i].tobytes()


def test_c1_first_call_generic_then_keyed_then_hit(kct):
    c = Cache(kct, 10_000)
    vals = keys(b"c1", 0, 175)
    (k1, _), = c.call([(vals, 175)])
    assert not k1  # 175 signatures cannot pay for 175 keys: generic now, built after the call
    s = c.stats()
    assert s["generic_sets"] == 1 and s["keys_deferred"] == 175 and s["pool_keys"] == 175 and s["pending_keys"] == 0
    (k2, idx2), = c.call([(vals, 175)])
    assert k2 and c.stats()["hits"] == 0  # every key pooled: keyed at once, entry created
    check_idx(c, vals, idx2)
    (k3, idx3), = c.call([(vals, 175)])
    assert k3 and c.stats()["hits"] == 1 and (idx3 == idx2).all()
    assert c.stats()["keys_appended"] == 175  # nothing rebuilt
    c.close()


def test_large_call_builds_its_keys_first(kct):
    c = Cache(kct, 100_000)
    vals = keys(b"c4", 0, 1000)
    (k, idx), = c.call([(vals, AMORTIZE * 1000)])  # a blocksync window: its signatures pay for every key
    assert k and c.stats()["keys_deferred"] == 0 and c.stats()["keys_appended"] == 1000
    check_idx(c, vals, idx)
    (k, _), = c.call([(vals, AMORTIZE * 1000 - 1)], force=False)
    assert k and c.stats()["hits"] == 1


def test_light_client_sets_share_pooled_keys(kct):
    """Sets of 175 changing one key per height (the C3 chain): after the cold call the pool holds
    each key once; a later batch of 50 sets is keyed with at most one build per new key."""
    c = Cache(kct, 100_000)
    pool = keys(b"c3", 0, 300)
    sets = [pool[h:h + 175] for h in range(60)]
    res = c.call([(s, 176) for s in sets[:50]])
    assert not any(k for k, _ in res)                      # cold: generic, keys built after the call
    assert c.stats()["pool_keys"] == 50 + 174               # each distinct key once
    res = c.call([(s, 176) for s in sets[:50]])
    assert all(k for k, _ in res)
    for s, (_, idx) in zip(sets[:50], res):
        check_idx(c, s, idx)
    # ten more heights: one new key each; the call is small, so those ten sets stay generic once
    res = c.call([(s, 176) for s in sets[40:60]])
    assert [k for k, _ in res] == [True] * 10 + [False] * 10
    assert c.stats()["pool_keys"] == 60 + 174
    res = c.call([(s, 176) for s in sets[40:60]])
    assert all(k for k, _ in res)


def test_call_level_amortisation(kct):
    """A call is keyed when its signatures pay for ALL its missing keys, even if one set alone
    would not (commit.hip keycache_resolve: build_all)."""
    c = Cache(kct, 100_000)
    pool = keys(b"am", 0, 400)
    sets = [pool[h:h + 100] for h in range(0, 300, 100)]
    miss = sum(kct.kct_missing(c.h, np.ascontiguousarray(s).ctypes.data, len(s)) for s in sets)
    assert miss == 300
    res = c.call([(s, 10) for s in sets], force=True)  # the seam's decision for call_sigs >= 2048 * 300
    assert all(k for k, _ in res) and c.stats()["keys_deferred"] == 0


def test_budget_reset_and_pinning(kct):
    c = Cache(kct, 300)
    a, b = keys(b"A", 0, 175), keys(b"B", 0, 175)
    assert c.call([(a, AMORTIZE * 175)])[0][0]
    # another call in flight holds indexes into the pool: B cannot reset it, stays generic
    kct.kct_pin(c.h)
    k, _ = c.call([(b, AMORTIZE * 175)])[0]
    assert not k and c.stats()["pool_resets"] == 0
    kct.kct_unpin(c.h)
    k, idx = c.call([(b, AMORTIZE * 175)])[0]
    assert k and c.stats()["pool_resets"] == 1 and c.stats()["pool_keys"] == 175
    check_idx(c, b, idx)
    # A was dropped with the pool: a miss again (generic when small)
    k, _ = c.call([(a, 175)])[0]
    assert not k
    # a set larger than the whole budget is never keyed
    big = keys(b"big", 0, 301)
    assert not c.call([(big, AMORTIZE * 1000)])[0][0]


def test_hit_is_compared_key_by_key(kct):
    """The same set_hash for two different key lists (a stale or wrong hash, a digest collision)
    costs a miss; the indexes always name the set's own keys."""
    c = Cache(kct, 10_000)
    h = hashlib.sha256(b"ValidatorSet.Hash").digest()
    a, b = keys(b"hA", 0, 50), keys(b"hB", 0, 50)
    k, ia = c.lookup(a, AMORTIZE * 50, set_hash=h, force=True)
    assert k
    check_idx(c, a, ia)
    k, ib = c.lookup(b, AMORTIZE * 50, set_hash=h, force=True)
    assert k and c.stats()["hits"] == 0
    check_idx(c, b, ib)
    k, ia2 = c.lookup(a, 50, set_hash=h)
    assert k and c.stats()["hits"] == 0  # entry holds b now; a's keys are pooled: keyed, not a hit
    check_idx(c, a, ia2)
    # the digest key (no set_hash) and the hash key are separate entries of the same keys
    k, ia3 = c.lookup(a, 50)
    assert k and (ia3 == ia2).all()


def test_repeated_keys_and_failed_builds(kct):
    c = Cache(kct, 10_000)
    a = keys(b"dup", 0, 20)
    a[7] = a[3]  # two validators with one key (cannot happen in Tendermint; must still be exact)
    k, idx = c.lookup(a, AMORTIZE * 20, force=True)
    assert k and idx[7] == idx[3] and c.stats()["pool_keys"] == 19
    check_idx(c, a, idx)
    kct.kct_fail_next_append(c.h)
    b = keys(b"fail", 0, 10)
    k, _ = c.lookup(b, AMORTIZE * 10, force=True)
    assert not k and c.stats()["pool_keys"] == 19  # a failed build leaves the set generic
    k, idx = c.lookup(b, AMORTIZE * 10, force=True)
    assert k
    check_idx(c, b, idx)


def test_entry_bounds_lru(kct):
    c = Cache(kct, 10_000)
    kct.kct_limits(c.h, 4, 1 << 30)
    sets = [keys(b"lru%d" % i, 0, 8) for i in range(6)]
    for s in sets:
        assert c.lookup(s, AMORTIZE * 8, force=True)[0]
    s = c.stats()
    assert s["sets_cached"] <= 4 and s["sets_evicted"] >= 2
    assert c.lookup(sets[-1], 8)[0] and c.stats()["hits"] == 1  # the most recent entry survives
    assert c.lookup(sets[0], 8)[0]  # evicted entry: keys still pooled, keyed again (not a hit)
    assert c.stats()["hits"] == 1


def test_entries_dropped_while_pinned_are_retired(kct):
    """A call resolves raw entry pointers (no reference count per set): entries the LRU bound, a
    key mismatch or a reset drop while any call is pinned are retired and freed at the last unpin."""
    c = Cache(kct, 10_000)
    kct.kct_limits(c.h, 2, 1 << 30)
    sets = [keys(b"ret%d" % i, 0, 8) for i in range(5)]
    kct.kct_pin(c.h)
    for s in sets:
        assert c.lookup(s, AMORTIZE * 8, force=True)[0]
    assert c.stats()["sets_evicted"] >= 2 and kct.kct_retired(c.h) == c.stats()["sets_evicted"]
    kct.kct_pin(c.h)    # a second call
    kct.kct_unpin(c.h)
    assert kct.kct_retired(c.h) > 0  # the first call is still pinned
    kct.kct_unpin(c.h)
    assert kct.kct_retired(c.h) == 0
    # unpinned: dropped entries are freed at once
    for s in sets:
        assert c.lookup(s, AMORTIZE * 8, force=True)[0]
    assert kct.kct_retired(c.h) == 0


def test_deferred_first_commit_of_a_new_set(kct):
    """The seam's fast path for a single commit on a new set (commit.hip keycache_resolve): one
    pool probe (all_pooled stops at the first missing key), the keys copied (defer), the call
    generic; the worker's drain then queues and builds exactly the missing keys, and the next
    commit on the set is keyed.  Counted as the deferred lookup path counts."""
    c = Cache(kct, 10_000)
    a = keys(b"df", 0, 175)
    assert c.call([(a[:100], AMORTIZE * 100)])[0][0]          # 100 of the keys pooled by a big call
    pa = np.ascontiguousarray(a)
    assert kct.kct_all_pooled(c.h, pa.ctypes.data, 175) == 0
    assert kct.kct_all_pooled(c.h, np.ascontiguousarray(a[:100]).ctypes.data, 100) == 1
    s0 = c.stats()
    kct.kct_pin(c.h)
    kct.kct_defer(c.h, pa.ctypes.data, 175, 175)
    kct.kct_unpin(c.h)
    s1 = c.stats()
    assert s1["generic_sets"] == s0["generic_sets"] + 1 and s1["lookups"] == s0["lookups"] + 1
    assert s1["pool_keys"] == 100                             # nothing looked up or built in the call
    assert kct.kct_drain(c.h) == 0
    s2 = c.stats()
    assert s2["pool_keys"] == 175 and s2["keys_deferred"] == s0["keys_deferred"] + 75
    k, idx = c.call([(a, 175)])[0]
    assert k
    check_idx(c, a, idx)


def test_digest_depends_on_order_and_size(kct):
    a = keys(b"dg", 0, 10)
    outs = set()
    for arr in (a, a[::-1].copy(), a[:9].copy()):
        o = ctypes.create_string_buffer(32)
        kct.kct_digest(np.ascontiguousarray(arr).ctypes.data, len(arr), o)
        outs.add(o.raw)
    assert len(outs) == 3
