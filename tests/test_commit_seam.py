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
