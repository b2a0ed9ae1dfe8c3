"""GPU parity of the opt-in ZIP-215 batch mode (tmed_verify_batch_zip215, csrc/zip215.hip).

Expected bits come from the ZIP-215 restatement — oracle/zip215.py (big integers) and the C port's
port_verify_zip215 — pinned against each other on tests/golden/zip215_vectors.json; the
reference holds no ZIP-215 code or vectors (spec/core/encoding.md:52-54 only names the rule), so
this parity is "derived from the ZIP-215 rule, unpinned by the reference".  Covered paths:
  * the randomized batch equation passing for a whole chunk (all valid, including the tuples
    ZIP-215 accepts and Go rejects: mixed-order R and A, non-canonical and negative-zero R,
    small-order A and R with S = 0) — one MSM, no single checks;
  * bisection down to groups decided signature by signature (one bad signature in 70k);
  * dense failures (the golden classes, the C5 mix) decided by the exact single check."""
import json
import os

import numpy as np
import pytest

from oracle import port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _zip_golden():
    base = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_vectors.json")))["vectors"]
    z = json.load(open(os.path.join(ROOT, "tests", "golden", "zip215_vectors.json")))
    out = []
    for v, ok in zip(base, z["base_valid_zip215"]):
        out.append((v["class"], bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), ok))
    for v in z["vectors"]:
        out.append((v["class"], bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]),
                    v["valid_zip215"]))
    return out


def _pack(items):
    n = len(items)
    pubs = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 64), np.uint8)
    lens = np.zeros(n, np.uint32)
    ms = []
    for i, (_, p, m, s, _) in enumerate(items):
        pubs[i] = np.frombuffer(p, np.uint8)
        sigs[i, :min(64, len(s))] = np.frombuffer(s[:64], np.uint8)
        lens[i] = len(s)
        ms.append(m)
    offs = np.zeros(n + 1, np.uint32)
    offs[1:] = np.cumsum([len(m) for m in ms])
    msgs = np.frombuffer(b"".join(ms) + b"\0" * 16, np.uint8)
    return pubs, sigs, lens, msgs, offs


def _signed_batch(engine, n, seed):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    offs = (np.arange(n + 1) * 114).astype(np.uint32)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = engine.sign_arrays(seeds, msgs, offs)
    return rng, pubs, sigs, msgs, offs


def test_golden_classes(engine):
    items = [it for it in _zip_golden() if len(it[1]) == 32]
    pubs, sigs, lens, msgs, offs = _pack(items)
    out = engine.verify_zip215_arrays(pubs, sigs, msgs, offs, lens)
    exp = np.array([it[4] for it in items], np.uint8)
    bad = [items[i][0] for i in np.nonzero(out != exp)[0]]
    assert not bad, bad[:20]
    # and the C port agrees with the fixtures on the same packing
    assert (port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 8, lens, zip215=True) == exp).all()


def test_batch_equation_accepts_zip215_edge_cases(engine):
    """50k valid signatures plus every golden tuple ZIP-215 accepts (mixed-order and small-order
    points, non-canonical R): one batch equation holds, no signature is decided singly."""
    rng, pubs, sigs, msgs, offs = _signed_batch(engine, 50_000, 215)
    acc = [it for it in _zip_golden() if it[4] == 1 and len(it[1]) == 32 and len(it[3]) == 64]
    assert len(acc) > 700
    ep, es, _, em, eo = _pack(acc)
    pubs = np.concatenate([pubs, ep])
    sigs = np.concatenate([sigs, es])
    msgs2 = np.concatenate([msgs[:int(offs[-1])], em])
    offs2 = np.concatenate([offs[:-1], eo + offs[-1]]).astype(np.uint32)
    perm = rng.permutation(pubs.shape[0])  # spread the edge tuples over the chunk
    lens = np.diff(offs2.astype(np.int64))
    starts = offs2[:-1].astype(np.int64)
    msgs3 = np.concatenate([msgs2[starts[i]:starts[i] + lens[i]] for i in perm] + [np.zeros(16, np.uint8)])
    offs3 = np.zeros(len(perm) + 1, np.uint32)
    offs3[1:] = np.cumsum(lens[perm])
    pubs, sigs = pubs[perm], sigs[perm]
    from tmed import Engine
    Engine.zip215_set_seed(bytes(range(32)))
    try:
        out = engine.verify_zip215_arrays(pubs, sigs, msgs3, offs3)
        st = Engine.zip215_stats()
    finally:
        Engine.zip215_set_seed(None)
    assert out.all(), int((out == 0).sum())
    assert st["equations"] == 1 and st["single_sigs"] == 0, st
    exp = port.verify_batch(pubs, sigs, msgs3, offs3.astype(np.uint64), 16, zip215=True)
    assert exp.all()


def test_bisection_finds_one_bad_signature(engine):
    from tmed import Engine
    rng, pubs, sigs, msgs, offs = _signed_batch(engine, 70_000, 7)
    bad = 52_345
    sigs[bad, 40] ^= 0x10
    out = engine.verify_zip215_arrays(pubs, sigs, msgs, offs)
    st = Engine.zip215_stats()
    exp = np.ones(70_000, np.uint8)
    exp[bad] = 0
    assert int((out != exp).sum()) == 0
    assert st["equations"] >= 3 and 0 < st["single_sigs"] < 70_000, st


@pytest.mark.parametrize("n", [1, 63, 1000, 20_000])
def test_random_flips_vs_port(engine, n):
    rng, pubs, sigs, msgs, offs = _signed_batch(engine, n, 100 + n)
    sigs[::9, int(rng.integers(0, 64))] ^= 0x02
    out = engine.verify_zip215_arrays(pubs, sigs, msgs, offs)
    exp = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16, zip215=True)
    assert int((out != exp).sum()) == 0


def test_c5_mix_vs_port(engine):
    from tmed.workload import c5_mix
    rng, pubs, sigs, msgs, offs = _signed_batch(engine, 100_000, 0x5EED)
    c5_mix(pubs, sigs, seed=0x5EED)
    out = engine.verify_zip215_arrays(pubs, sigs, msgs, offs)
    exp = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16, zip215=True)
    assert int((out != exp).sum()) == 0
    # the default (Go 1.18) path on the same tuples is unchanged and differs where the rules do
    go = engine.verify_arrays(pubs, sigs, msgs, offs)
    assert int((go != port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16)).sum()) == 0


def test_dense_failures_cut_off():
    """Failure cut-off (zip215.hip kZipSinglyMin): after a chunk with failures (the C5 mix: the
    equation and both halves fail), the next chunk is decided signature by signature with no MSM;
    its failures are counted on the device and a chunk without any puts the next one back on the
    batch equation.  Decisions equal the port's ZIP-215 bits on every call."""
    from conftest import engine_with_env
    from tmed import Engine
    from tmed.workload import c5_mix
    eng = engine_with_env()
    try:
        rng, pubs, sigs, msgs, offs = _signed_batch(eng, 70_000, 0xC5)
        good_p, good_s = pubs.copy(), sigs.copy()
        c5_mix(pubs, sigs, seed=0xC5)
        exp = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16, zip215=True)
        stats = []
        for _ in range(2):
            out = eng.verify_zip215_arrays(pubs, sigs, msgs, offs)
            stats.append(Engine.zip215_stats())
            assert int((out != exp).sum()) == 0
        assert stats[0]["equations"] == 3 and stats[0]["single_sigs"] == 70_000, stats
        assert stats[1]["equations"] == 0 and stats[1]["single_sigs"] == 70_000, stats
        out = eng.verify_zip215_arrays(good_p, good_s, msgs, offs)  # singly (its predecessor failed) ...
        st = Engine.zip215_stats()
        assert out.all() and st["equations"] == 0 and st["single_sigs"] == 70_000, st
        out = eng.verify_zip215_arrays(good_p, good_s, msgs, offs)  # ... and no failure: batch mode again
        st = Engine.zip215_stats()
        assert out.all() and st["equations"] == 1 and st["single_sigs"] == 0, st
        # one bad signature: bisection, then the next chunk singly, whose count (one) keeps it so
        one = good_s.copy()
        one[1234, 7] ^= 0x40
        exp1 = np.ones(70_000, np.uint8)
        exp1[1234] = 0
        for want_eq in (None, 0, 0):
            out = eng.verify_zip215_arrays(good_p, one, msgs, offs)
            st = Engine.zip215_stats()
            assert int((out != exp1).sum()) == 0
            if want_eq is None:
                assert st["equations"] >= 3 and st["single_sigs"] < 70_000, st
            else:
                assert st["equations"] == want_eq and st["single_sigs"] == 70_000, st
    finally:
        eng.close()


def test_failure_policy_across_chunks_of_one_call():
    """One call over several chunks (TMED_SLAB_SLOTS = 65,536: chunks of 65,536 signatures): the
    first half of the batch carries the C5 mix, the second half is all valid.  Chunk 0 runs the
    equation and bisects, chunk 1 (its predecessor failed) is decided singly and its failures are
    counted, chunk 2 — the first clean chunk — is decided singly too (chunk 1 had failures), and
    chunk 3 returns to the batch equation (chunk 2 counted none).  Decisions equal the port's."""
    from conftest import engine_with_env
    from tmed import Engine
    from tmed.workload import c5_mix
    eng = engine_with_env(TMED_SLAB_SLOTS=65536)
    try:
        n, half = 4 * 65536, 2 * 65536
        rng, pubs, sigs, msgs, offs = _signed_batch(eng, n, 0xC4C4)
        p, s = pubs[:half].copy(), sigs[:half].copy()
        c5_mix(p, s, seed=0xC4)
        pubs[:half], sigs[:half] = p, s
        exp = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16, zip215=True)
        assert int((exp[:65536] == 0).sum()) > 0 and int((exp[65536:half] == 0).sum()) > 0 and exp[half:].all()
        out = eng.verify_zip215_arrays(pubs, sigs, msgs, offs)
        st = Engine.zip215_stats()
        assert int((out != exp).sum()) == 0
        assert st["chunks"] == 4, st
        # chunk 0: the equation + its halves (dense), then chunks 1 and 2 singly, chunk 3 one equation
        assert st["single_sigs"] == 3 * 65536 and st["equations"] == 4, st
    finally:
        eng.close()
