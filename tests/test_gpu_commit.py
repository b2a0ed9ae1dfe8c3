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
