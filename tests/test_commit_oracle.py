"""Commit-loop restatement vs the reference's own decision/error cases.

types/validator_set_test.go:670-744 (VerifyCommit_All), :746-769 (CheckAllSignatures),
:771-792 (Light returns early), :794-815 (Trusting returns early), :1520-1559
(Trusting overlap), :1561-1574 (int64 overflow).
"""
import pytest

from oracle import commit as C
from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of


def _vs(n, power, tag="v"):
    return make_valset([seed_of(tag, i) for i in range(n)], [power] * n)


def test_verify_commit_all():
    vs, seeds = _vs(1, 1000, "all")
    chain = "Lalande21185"
    bid = make_block_id("all")
    commit = make_commit(vs, seeds, chain, 12345, 2, bid)
    h = 12345
    cases = [
        ("good", chain, bid, h, commit, None),
        ("wrong signature (#0)", "EpsilonEridani", bid, h, commit, "wrong signature (#0)"),
        ("wrong block ID", chain, make_block_id("other"), h, commit, "wrong block ID"),
        ("wrong height", chain, bid, h - 1, commit, "wrong height"),
        ("1 vs 0", chain, bid, h, C.Commit(h, 2, bid, []), "wrong set size: 1 vs 0"),
        ("1 vs 2", chain, bid, h, C.Commit(h, 2, bid, [commit.signatures[0], C.CommitSig(C.FLAG_ABSENT)]),
         "wrong set size: 1 vs 2"),
        ("power", chain, bid, h, C.Commit(h, 2, bid, [C.CommitSig(C.FLAG_ABSENT)]),
         "insufficient voting power: got 0, needed more than 666"),
    ]
    c2 = make_commit(vs, seeds, chain, h, 2, bid)
    resign(c2, 0, seeds[0], "EpsilonEridani")
    cases.append(("sig2", chain, bid, h, c2, "wrong signature (#0)"))
    for name, cid, b, hh, cm, exp in cases:
        for fn in (C.verify_commit, C.verify_commit_light):
            err = fn(vs, cid, b, hh, cm)
            if exp is None:
                assert err is None, (name, err)
            else:
                assert err is not None and exp in str(err), (name, str(err))


def test_error_types_and_text():
    vs, seeds = _vs(1, 1000, "t")
    bid = make_block_id("t")
    cm = make_commit(vs, seeds, "c", 3, 0, bid)
    e = C.verify_commit(vs, "c", bid, 4, cm)
    assert isinstance(e, C.ErrInvalidCommitHeight) and str(e) == "Invalid commit -- wrong height: 4 vs 3"
    e = C.verify_commit(vs, "c", bid, 3, C.Commit(3, 0, bid, []))
    assert isinstance(e, C.ErrInvalidCommitSignatures) and str(e) == "Invalid commit -- wrong set size: 1 vs 0"
    e = C.verify_commit(vs, "c", make_block_id("x"), 3, cm)
    assert str(e).startswith("invalid commit -- wrong block ID: want ")
    e = C.verify_commit(vs, "d", bid, 3, cm)
    assert str(e) == "wrong signature (#0): " + cm.signatures[0].signature.hex().upper()


def test_check_all_signatures_and_light_early_exit():
    vs, seeds = _vs(4, 10, "chk")
    bid = make_block_id("chk")
    cm = make_commit(vs, seeds, "test_chain_id", 3, 0, bid)
    resign(cm, 3, seeds[3], "CentaurusA")
    assert "wrong signature (#3)" in str(C.verify_commit(vs, "test_chain_id", bid, 3, cm))
    assert C.verify_commit_light(vs, "test_chain_id", bid, 3, cm) is None


def test_trusting_early_exit():
    vs, seeds = _vs(4, 10, "tr")
    bid = make_block_id("tr")
    cm = make_commit(vs, seeds, "test_chain_id", 3, 0, bid)
    resign(cm, 2, seeds[2], "CentaurusA")
    assert C.verify_commit_light_trusting(vs, "test_chain_id", cm, 1, 3) is None


def test_trusting_overlap():
    vs, seeds = _vs(6, 1, "ov")
    bid = make_block_id("ov")
    cm = make_commit(vs, seeds, "test_chain_id", 1, 1, bid)
    new_vs, _ = _vs(2, 1, "ov-new")
    assert C.verify_commit_light_trusting(vs, "test_chain_id", cm, 1, 3) is None
    e = C.verify_commit_light_trusting(new_vs, "test_chain_id", cm, 1, 3)
    assert isinstance(e, C.ErrNotEnoughVotingPowerSigned) and e.got == 0
    merged = C.ValidatorSet(new_vs.validators + vs.validators)
    assert C.verify_commit_light_trusting(merged, "test_chain_id", cm, 1, 3) is None


def test_trusting_overflow_and_zero_den():
    vs, seeds = _vs(1, C.MAX_TOTAL_VOTING_POWER, "of")
    bid = make_block_id("of")
    cm = make_commit(vs, seeds, "test_chain_id", 1, 1, bid)
    assert "int64 overflow" in str(C.verify_commit_light_trusting(vs, "test_chain_id", cm, 25, 55))
    assert str(C.verify_commit_light_trusting(vs, "test_chain_id", cm, 1, 0)) == "trustLevel has zero Denominator"


def test_trusting_double_vote():
    vs, seeds = _vs(3, 10, "dv")
    bid = make_block_id("dv")
    cm = make_commit(vs, seeds, "test_chain_id", 5, 0, bid)
    cm.signatures[2].address = cm.signatures[0].address
    e = C.verify_commit_light_trusting(vs, "test_chain_id", cm, 2, 3)
    assert str(e).startswith("double vote from Validator{") and str(e).endswith("(0 and 2)")


def test_nil_votes_verified_but_not_tallied():
    vs, seeds = _vs(4, 10, "nil")
    bid = make_block_id("nil")
    flags = [C.FLAG_COMMIT, C.FLAG_NIL, C.FLAG_COMMIT, C.FLAG_COMMIT]
    cm = make_commit(vs, seeds, "c", 7, 0, bid, flags=flags)
    assert C.verify_commit(vs, "c", bid, 7, cm) is None       # 30 > 26
    resign(cm, 1, seeds[1], "zzz")                             # a bad nil vote fails VerifyCommit...
    assert "wrong signature (#1)" in str(C.verify_commit(vs, "c", bid, 7, cm))
    assert C.verify_commit_light(vs, "c", bid, 7, cm) is None  # ...but Light never looks at it
    flags = [C.FLAG_COMMIT, C.FLAG_NIL, C.FLAG_NIL, C.FLAG_ABSENT]
    cm = make_commit(vs, seeds, "c", 7, 0, bid, flags=flags)
    e = C.verify_commit(vs, "c", bid, 7, cm)
    assert isinstance(e, C.ErrNotEnoughVotingPowerSigned) and (e.got, e.needed) == (10, 26)
