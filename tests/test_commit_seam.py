"""The C++ commit seam (plan -> one batch -> replay, csrc/commit.hip) reproduces the
reference loops' decisions and error values exactly.  CPU: the batch verifier is the
oracle (tmed_verify_commits_with); the GPU run of the same scenarios is in
tests/test_gpu_commit.py."""
import numpy as np

from oracle import port
from commit_cases import oracle_result, pbid, same, scenarios
import tmed.types as T


def oracle_verifier(pubs, sigs, lens, msgs, offs):
    out = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 4)
    out[lens != 64] = 0
    return out


def test_seam_matches_reference_loops_cpu():
    reqs, exp = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=1, count=80):
        exp.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    # one batch for all requests, and one request at a time
    got_batch = T.verify_commits(None, reqs, verifier=oracle_verifier)
    for q, r in enumerate(reqs):
        got_one = T.verify_commits(None, [r], verifier=oracle_verifier)[0]
        assert same(got_one, exp[q]), (q, got_one, exp[q])
        assert same(got_batch[q], exp[q]), (q, got_batch[q], exp[q])
    kinds = {type(e).__name__ if e is not None else "ok" for e in exp}
    assert {"ok", "GoError", "ErrNotEnoughVotingPowerSigned"} <= kinds


def test_light_verifies_only_the_prefix():
    from oracle.fixtures import make_block_id, make_commit, make_valset, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("pfx", i) for i in range(30)], [10] * 30)
    bid = make_block_id("pfx")
    cm = make_commit(vs, seeds, "c", 9, 0, bid)
    pv, pc = to_product(vs, cm)
    stats = []
    errs = T.verify_commits(None, [(T.MODE_LIGHT, pv, "c", pbid(bid), 9, pc, 0, 0),
                                   (T.MODE_COMMIT, pv, "c", pbid(bid), 9, pc, 0, 0),
                                   (T.MODE_LIGHT_TRUSTING, pv, "c", None, 0, pc, 1, 3)],
                            verifier=oracle_verifier, stats=stats)
    assert errs == [None, None, None]
    assert stats == [21, 30, 11]  # > 2/3 of 300 after 21 sigs; all 30; > 1/3 after 11


def test_parallel_plan_and_replay_equal_serial():
    """Batches above 65,536 signatures are planned and replayed on host threads; the result
    of every request must equal its result as a single (serial) call.  The verifier is a
    deterministic stand-in (bit = low bit of sig[1]) so the test needs no signing."""
    rng = np.random.default_rng(3)
    n_vals, n_req = 150, 480
    pubs = rng.integers(0, 256, (n_vals, 32), dtype=np.uint8)
    vals = T.ValidatorSet([T.Validator(bytes(p), int(w), 0) for p, w in zip(pubs, rng.integers(1, 50, n_vals))])
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    reqs = []
    for q in range(n_req):
        flags = rng.choice(np.array([1, 2, 2, 2, 2, 3], np.uint8), n_vals)
        sigs = rng.integers(0, 256, (n_vals, 64), dtype=np.uint8)
        sigs[:, 1] |= (rng.random(n_vals) < 0.97).astype(np.uint8)  # ~3% invalid
        bid = T.BlockID(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), 3,
                        bytes(rng.integers(0, 256, 32, dtype=np.uint8)))
        ad = addrs.copy()
        if q % 5 == 4:
            ad[7] = ad[3]                                        # double vote for Trusting
        pc = T.PackedCommit(10 + q, 0, bid, flags, ad, np.full(n_vals, 1700000000 + q, np.int64),
                            np.zeros(n_vals, np.int32), sigs, np.full(n_vals, 64, np.uint32))
        mode = q % 3
        reqs.append((mode, vals, "par", bid if mode != 2 else None, 10 + q, pc, 1, 3))

    def bitfn(pubs_, sigs_, lens, msgs, offs):
        return (sigs_[:, 1] & 1).astype(np.uint8)

    got = T.verify_commits(None, reqs, verifier=bitfn)
    assert sum(int(reqs[q][5].flags.shape[0]) for q in range(n_req)) >= 65536
    for q in range(0, n_req, 3):
        one = T.verify_commits(None, [reqs[q]], verifier=bitfn)[0]
        assert same(got[q], one), (q, got[q], one)
    assert len({type(e).__name__ for e in got}) >= 2


def _one_commit(flag_override=None):
    from oracle.fixtures import make_block_id, make_commit, make_valset, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("ei", i) for i in range(4)], [10] * 4)
    bid = make_block_id("ei")
    cm = make_commit(vs, seeds, "ei-chain", 7, 0, bid)
    pv, pc = to_product(vs, cm)
    if flag_override is not None:
        pc.signatures[2].flag = flag_override
    return vs, pv, cm, pc, bid


def test_inputs_the_reference_panics_on_return_einval():
    """Where the reference would panic — an unknown BlockIDFlag reaching CommitSig.BlockID
    (types/block.go:652-662) in VerifyCommit — the seam returns TMED_EINVAL so the caller takes
    the original Go path (which then panics exactly as before); an unknown flag in the Light
    loops is skipped like any non-Commit flag, as the reference does (validator_set.go:742)."""
    import pytest
    from tmed import TmedError
    from tmed._native import TMED_EINVAL
    vs, pv, cm, pc, bid = _one_commit(flag_override=9)
    with pytest.raises(TmedError) as ei:
        T.verify_commits(None, [(T.MODE_COMMIT, pv, "ei-chain", pbid(bid), 7, pc, 0, 0)], verifier=oracle_verifier)
    assert ei.value.code == TMED_EINVAL
    # Light: flag 9 is not BlockIDFlagCommit -> skipped; 3 of 4 equal powers still cross 2/3
    got = T.verify_commits(None, [(T.MODE_LIGHT, pv, "ei-chain", pbid(bid), 7, pc, 0, 0)], verifier=oracle_verifier)
    assert got == [None]


def test_bad_mode_and_missing_block_id_return_einval():
    import pytest
    from tmed import TmedError
    vs, pv, cm, pc, bid = _one_commit()
    with pytest.raises(TmedError):
        T.verify_commits(None, [(7, pv, "ei-chain", pbid(bid), 7, pc, 0, 0)], verifier=oracle_verifier)
    with pytest.raises(TmedError):  # VerifyCommit / Light need a BlockID
        T.verify_commits(None, [(T.MODE_LIGHT, pv, "ei-chain", None, 7, pc, 0, 0)], verifier=oracle_verifier)
