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


def test_trusting_first_match_with_duplicate_addresses():
    """GetByAddress returns the FIRST validator with the address (types/validator_set.go:270-277).
    The planner tries signature i's own position first; in a set where validator 2's address also
    sits at position 0, signature 2 must still map to validator 0 — a double vote when signature
    0 carries the same address."""
    from oracle import commit as C
    from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of
    from commit_cases import to_product
    vs, seeds = make_valset([seed_of("dupa", i) for i in range(6)], [10, 20, 30, 40, 50, 60])
    bid = make_block_id("dupa")
    reqs, exp = [], []
    for absent0 in (False, True):
        flags = [C.FLAG_ABSENT if (absent0 and i == 0) else C.FLAG_COMMIT for i in range(6)]
        cm = make_commit(vs, seeds, "c", 5, 0, bid, flags=flags)
        if not absent0:  # signature 0 carries validator 2's address: both map to validator 0
            cm.signatures[0].address = vs.validators[2].address
            resign(cm, 0, seeds[2], "c")  # ... and validator 2's signature
        tvs = C.ValidatorSet([vs.validators[2]] + vs.validators[1:])
        for num, den in ((1, 3), (2, 3), (1, 1)):
            exp.append(C.verify_commit_light_trusting(tvs, "c", cm, num, den))
            pv, pc = to_product(tvs, cm)
            reqs.append((T.MODE_LIGHT_TRUSTING, pv, "c", None, 0, pc, num, den))
    got = T.verify_commits(None, reqs, verifier=oracle_verifier)
    for q in range(len(reqs)):
        assert same(got[q], exp[q]), (q, got[q], exp[q])
    assert any(e is not None and "double vote" in str(e) for e in exp)


def test_parallel_plan_and_replay_equal_serial():
    """Batches above 65,536 signatures are planned and replayed on host threads (and calls of
    more than 1,024 requests check them on host threads); the result of every request must equal
    its result as a single (serial) call.  Each Trusting request shares the commit of the Light
    request before it (the light client's pair: the seam's candidate aliasing and shared
    templates run).  The verifier is a deterministic stand-in (bit = low bit of sig[1]) so the
    test needs no signing."""
    rng = np.random.default_rng(3)
    n_vals, n_req = 150, 1100
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
        if mode == 2:  # Trusting on the Light request's commit
            pc, bid = reqs[-1][5], reqs[-1][3]
        reqs.append((mode, vals, "par", bid if mode != 2 else None, 10 + q, pc, 1, 3))

    def bitfn(pubs_, sigs_, lens, msgs, offs):
        return (sigs_[:, 1] & 1).astype(np.uint8)

    got = T.verify_commits(None, reqs, verifier=bitfn)
    assert sum(int(reqs[q][5].flags.shape[0]) for q in range(n_req)) >= 65536
    for q in list(range(0, n_req, 7)) + list(range(2, n_req, 9)):
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


def test_inputs_the_reference_panics_on_are_per_request():
    """Where the reference loop would panic — an unknown BlockIDFlag reaching CommitSig.BlockID
    (types/block.go:652-665) in VerifyCommit — the request gets TMED_COMMIT_PANIC at that index
    (the Go shim then runs the original method, which panics exactly as before) — but only if the
    loop gets that far: a bad signature before it is reported as such.  An unknown flag in the
    Light loops is skipped like any non-Commit flag, as the reference does (validator_set.go:742).
    Other requests of the same batch are unaffected."""
    import pytest
    vs, pv, cm, pc, bid = _one_commit(flag_override=9)
    good = (T.MODE_COMMIT, *_one_commit()[1:2], "ei-chain", pbid(bid), 7, _one_commit()[3], 0, 0)
    got = T.verify_commits(None, [(T.MODE_COMMIT, pv, "ei-chain", pbid(bid), 7, pc, 0, 0), good],
                           verifier=oracle_verifier)
    assert isinstance(got[0], T.GoPanic) and got[0].idx == 2
    assert got[1] is None
    with pytest.raises(T.GoPanic):
        T._raise_panic(got[0])
    # a bad signature at index 1 comes first: the reference returns "wrong signature (#1)"
    s = bytearray(pc.signatures[1].signature)
    s[0] ^= 1
    pc.signatures[1].signature = bytes(s)
    got = T.verify_commits(None, [(T.MODE_COMMIT, pv, "ei-chain", pbid(bid), 7, pc, 0, 0)], verifier=oracle_verifier)
    assert str(got[0]).startswith("wrong signature (#1)")
    # Light: flag 9 is not BlockIDFlagCommit -> skipped; 3 of 4 equal powers still cross 2/3
    vs, pv, cm, pc, bid = _one_commit(flag_override=9)
    got = T.verify_commits(None, [(T.MODE_LIGHT, pv, "ei-chain", pbid(bid), 7, pc, 0, 0)], verifier=oracle_verifier)
    assert got == [None]


def test_edge_scenarios_match_reference_loops_cpu():
    """Unknown flags, malformed BlockID hashes and ValidatorAddress lengths 0/19/21 (including
    the 19-byte prefix of an address ending in 0x00) through the seam vs the oracle loops —
    panics reported per request at the reference's index, addresses matched by bytes.Equal."""
    from commit_cases import edge_scenarios, oracle_outcome, same_outcome
    reqs, exp = [], []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in edge_scenarios(seed=7, count=60):
        exp.append(oracle_outcome(mode, vs, chain, bid, h, cm, num, den))
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
    got = T.verify_commits(None, reqs, verifier=oracle_verifier)
    bad = [(q, got[q], exp[q]) for q in range(len(reqs)) if not same_outcome(got[q], exp[q])]
    assert not bad, bad[:5]
    kinds = {"panic" if isinstance(e, tuple) else (type(e).__name__ if e is not None else "ok") for e in exp}
    assert {"panic", "ok"} <= kinds, kinds


def test_address_prefix_of_zero_ending_address_is_not_a_match():
    """A ForBlock CommitSig whose ValidatorAddress is the 19-byte prefix of a validator address
    ending in 0x00 must be skipped by LightTrusting (bytes.Equal, types/validator_set.go:270-277):
    with the signature otherwise valid the tally lacks that validator's power."""
    from oracle import commit as C
    from oracle.fixtures import make_block_id, make_commit, make_valset, seed_of
    from commit_cases import address_ending_in_zero, oracle_outcome, to_product
    zs, zp = address_ending_in_zero()
    vs, seeds = make_valset([zs, seed_of("zp", 1), seed_of("zp", 2)], [10, 10, 10])
    cm = make_commit(vs, seeds, "zc", 5, 0, make_block_id("zc"))
    zi = next(i for i, v in enumerate(vs.validators) if v.pub_key == zp)
    assert vs.validators[zi].address[19] == 0
    cm.signatures[zi].address = vs.validators[zi].address[:19]
    exp = oracle_outcome(2, vs, "zc", None, 0, cm, 2, 3)
    pv, pc = to_product(vs, cm)
    got = T.verify_commits(None, [(T.MODE_LIGHT_TRUSTING, pv, "zc", None, 0, pc, 2, 3)], verifier=oracle_verifier)[0]
    assert str(got) == str(exp) == "invalid commit -- insufficient voting power: got 20, needed more than 20"
    # the bytes a fixed 20-byte slot holds for that address ARE the validator's address: only the
    # length crossing the ABI (address_lens) keeps them apart
    n = len(pc.signatures)
    addrs = np.zeros((n, 20), np.uint8)
    for i, cs in enumerate(pc.signatures):
        addrs[i, :len(cs.address[:20])] = np.frombuffer(cs.address[:20], np.uint8)
    assert addrs[zi].tobytes() == vs.validators[zi].address
    packed = T.PackedCommit(pc.height, pc.round, pc.block_id, np.array([s.flag for s in pc.signatures], np.uint8),
                            addrs, np.array([s.timestamp[0] for s in pc.signatures], np.int64),
                            np.array([s.timestamp[1] for s in pc.signatures], np.int32),
                            np.array([np.frombuffer(s.signature, np.uint8) for s in pc.signatures]),
                            np.full(n, 64, np.uint32),
                            np.array([len(s.address) for s in pc.signatures], np.uint32))
    got = T.verify_commits(None, [(T.MODE_LIGHT_TRUSTING, pv, "zc", None, 0, packed, 2, 3)], verifier=oracle_verifier)[0]
    assert str(got) == str(exp)
    packed.address_lens = None  # all 20: now the prefix slot matches, as a 20-byte shim would make it
    got = T.verify_commits(None, [(T.MODE_LIGHT_TRUSTING, pv, "zc", None, 0, packed, 2, 3)], verifier=oracle_verifier)[0]
    assert got is None


def test_bad_mode_and_missing_block_id_return_einval():
    import pytest
    from tmed import TmedError
    vs, pv, cm, pc, bid = _one_commit()
    with pytest.raises(TmedError):
        T.verify_commits(None, [(7, pv, "ei-chain", pbid(bid), 7, pc, 0, 0)], verifier=oracle_verifier)
    with pytest.raises(TmedError):  # VerifyCommit / Light need a BlockID
        T.verify_commits(None, [(T.MODE_LIGHT, pv, "ei-chain", None, 7, pc, 0, 0)], verifier=oracle_verifier)


def test_safe_mul_wraps_like_go():
    """safeMul (types/validator_set.go:1086-1105) with Go's int64 wrapping: a trust-level Numerator of
    2^63 reaches safeMul as int64 MinInt64, whose negation is MinInt64 again, so MaxInt64 / |b| is 0
    and any non-zero total power overflows (VERDICT r2 hygiene).  Oracle values are Go's by hand;
    the seam (csrc/commit.hip safe_mul) must give the same error for that request."""
    from oracle import commit as C
    MIN = -(1 << 63)
    assert C.safe_mul(10, MIN) == (0, True)
    assert C.safe_mul(MIN, 1) == (MIN, False)   # |MinInt64| wraps negative: no overflow, product -2^63
    assert C.safe_mul(MIN, -1) == (MIN, False)  # Go: MinInt64 * -1 wraps to MinInt64
    assert C.safe_mul(3, -4) == (-12, False)
    assert C.safe_mul(1 << 62, 2) == (0, True)
    assert C.safe_mul(0, MIN) == (0, False)
    vs, pv, cm, pc, bid = _one_commit()
    exp = C.verify_commit_light_trusting(vs, "ei-chain", cm, MIN, 3)
    assert "int64 overflow" in str(exp)
    got = T.verify_commits(None, [(T.MODE_LIGHT_TRUSTING, pv, "ei-chain", None, 0, pc, MIN, 3)],
                           verifier=oracle_verifier)[0]
    assert same(got, exp), (got, exp)


def test_edge_sign_bytes_host_encoder_cpu():
    """The commits of tests/test_gpu_signbytes_edges.py (zero time.Time, epoch, nanos 999,999,999,
    negative seconds, psh_total >= 2^28, heights >= 2^56, round 2^31-1, empty / 50 / 120 / 140-byte
    chain IDs, Nil and Absent flags) through the seam with the host-side encoder (csrc/signbytes.hip
    via tmed_verify_commits_with): equal to the oracle loops, the control commit included."""
    from test_gpu_signbytes_edges import _requests
    reqs, exp, _ = _requests(None)
    got = T.verify_commits(None, reqs, verifier=oracle_verifier)
    bad = [(q, str(g), str(e)) for q, (g, e) in enumerate(zip(got, exp)) if not same(g, e)]
    assert not bad, bad
