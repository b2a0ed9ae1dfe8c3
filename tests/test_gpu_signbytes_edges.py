"""Device CanonicalVote assembly at the edge encodings, through the commit seam.

Every signature is made by the oracle's signer over the ORACLE's sign-bytes
(oracle/signbytes.py, pinned by the 5 byte vectors of types/vote_test.go:60-137), and the seam
rebuilds the message on the device from a per-commit template plus the vote's flag and timestamp
(csrc/votes_dev.h assemble_vote, types/canonical.go:56-65, canonical.pb.go:517-579).  One wrong
byte of the device message turns that valid signature invalid, so VerifyCommit (which checks
every non-absent signature, Commit AND Nil flags: types/validator_set.go:685-700) must equal the
oracle loop on every commit.  Three device assemblers are exercised:
  * the generic latency kernel's hash lanes (verify_glat_prep_kernel, small batches);
  * the key-cached latency kernel's comb lanes (verify_keyset_lat_kernel);
  * assemble_votes_kernel in front of the throughput kernels (TMED_GLAT_MAX=0, TMED_LAT_MAX=0),
    generic and key-cached.
Edge encodings: the zero time.Time (seconds -62135596800: a 10-byte varint, vote_test.go:66-70),
the Unix epoch (both timestamp fields omitted), nanos 999,999,999, negative seconds with nanos,
year 9999, psh_total >= 2^28 (a 5-byte varint), heights >= 2^56, round 2^31 - 1, height 0 and
round 0 (fields omitted), an empty and a 50-byte chain ID (the genesis maximum,
types/genesis.go:21), Nil and Absent flags; a 120-byte chain ID still takes the device template
and a 140-byte one the host-assembled path (its longest message would overflow the 256-byte
device vote slot).  A generic tmed_verify_batch case with 1-4 KB messages covers the SHA-512
block loop past the vote sizes."""
import numpy as np
import pytest

from commit_cases import oracle_result, pbid, same, to_product
from conftest import engine_with_env
from oracle import commit as C
from oracle import port
from oracle.fixtures import make_valset, seed_of
import tmed.types as T

pytestmark = pytest.mark.gpu

STAMPS = [(-62135596800, 0), (0, 0), (1672531200, 999_999_999), (-1, 999_999_999), (253402300799, 999_999_999),
          (1, 1), (-62135596800, 1), (1 << 31, 0), (1672531200, 0), (0, 500)]

COMMITS = [  # chain, height, round, psh_total, flags
    ("test_chain_id", (1 << 56) + 5, 7, (1 << 28) + 3, None),
    ("e" * 49 + "Z", 1, (1 << 31) - 1, 1, None),
    ("", 0, 0, 123, None),
    ("x" * 120, (1 << 62) + 1, 3, (1 << 32) - 1, None),
    ("y" * 140, 77, 1, 123, None),
    ("test_chain_id", 9, 0, 123, [C.FLAG_NIL] * 3 + [C.FLAG_COMMIT] * 9),
]


def _edge_commit(k, chain, height, round_, psh_total, flags, n=12):
    vs, seeds = make_valset([seed_of("sbe%d" % k, i) for i in range(n)], [10] * n)
    bid = C.BlockID(bytes([k + 1]) * 32, psh_total, bytes([k + 101]) * 32)
    if flags is None:  # 9 Commit, 2 Nil, 1 Absent: > 2/3 of the power signs for the block
        flags = [C.FLAG_COMMIT, C.FLAG_NIL, C.FLAG_COMMIT, C.FLAG_ABSENT, C.FLAG_COMMIT, C.FLAG_COMMIT,
                 C.FLAG_NIL, C.FLAG_COMMIT, C.FLAG_COMMIT, C.FLAG_COMMIT, C.FLAG_COMMIT, C.FLAG_COMMIT]
    sigs = []
    cm = C.Commit(height, round_, bid, sigs)
    for i, v in enumerate(vs.validators):
        if flags[i] == C.FLAG_ABSENT:
            sigs.append(C.CommitSig(C.FLAG_ABSENT))
            continue
        sigs.append(C.CommitSig(flags[i], v.address, STAMPS[(i + k) % len(STAMPS)], b""))
        sigs[-1].signature = port.sign(seeds[i], cm.vote_sign_bytes(chain, i))
    return vs, cm, bid


def _requests(keyed_engine=None):
    reqs, exp, handles = [], [], []
    for k, (chain, h, r, pt, fl) in enumerate(COMMITS):
        vs, cm, bid = _edge_commit(k, chain, h, r, pt, fl)
        pv, pc = to_product(vs, cm)
        if keyed_engine is not None:
            pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators])
            pv.keyset = keyed_engine.keyset_load(pubs)
            pv.keyset_index = np.arange(len(pubs), dtype=np.uint32)
            handles.append(pv.keyset)
        exp.append(oracle_result(0, vs, chain, bid, h, cm, 0, 0))
        reqs.append((T.MODE_COMMIT, pv, chain, pbid(bid), h, pc, 0, 0))
    # the control: one Nil vote signed over the Commit-flag bytes must fail (the test can see a wrong byte)
    vs, cm, bid = _edge_commit(99, "test_chain_id", 5, 0, 123, None)
    nil_i = next(i for i, s in enumerate(cm.signatures) if s.flag == C.FLAG_NIL)
    cm.signatures[nil_i].flag = C.FLAG_COMMIT
    vs2, seeds2 = make_valset([seed_of("sbe99", i) for i in range(12)], [10] * 12)
    cm.signatures[nil_i].signature = port.sign(seeds2[nil_i], cm.vote_sign_bytes("test_chain_id", nil_i))
    cm.signatures[nil_i].flag = C.FLAG_NIL
    pv, pc = to_product(vs, cm)
    if keyed_engine is not None:
        pubs = np.array([np.frombuffer(v.pub_key, np.uint8) for v in pv.validators])
        pv.keyset = keyed_engine.keyset_load(pubs)
        pv.keyset_index = np.arange(len(pubs), dtype=np.uint32)
        handles.append(pv.keyset)
    exp.append(oracle_result(0, vs, "test_chain_id", bid, 5, cm, 0, 0))
    reqs.append((T.MODE_COMMIT, pv, "test_chain_id", pbid(bid), 5, pc, 0, 0))
    assert exp[-1] is not None and str(exp[-1]).startswith("wrong signature (#%d)" % nil_i)
    assert all(e is None for e in exp[:-1]), [str(e) for e in exp]
    return reqs, exp, handles


def _check(eng, keyed):
    reqs, exp, handles = _requests(eng if keyed else None)
    try:
        # all commits in one call, and each commit alone (one template per call)
        got = T.verify_commits(eng, reqs)
        bad = [(q, str(g), str(e)) for q, (g, e) in enumerate(zip(got, exp)) if not same(g, e)]
        assert not bad, bad
        for q, r in enumerate(reqs):
            g = T.verify_commits(eng, [r])[0]
            assert same(g, exp[q]), (q, str(g), str(exp[q]))
    finally:
        for h in handles:
            eng.keyset_free(h)


@pytest.fixture(scope="module")
def throughput_engine():
    e = engine_with_env(TMED_GLAT_MAX=0, TMED_LAT_MAX=0)
    yield e
    e.close()


@pytest.mark.parametrize("keyed", [False, True])
def test_edge_votes_latency_kernels(engine, keyed):
    """Generic: verify_glat_prep_kernel's in-lane assembly; keyed: verify_keyset_lat_kernel's."""
    _check(engine, keyed)


@pytest.mark.parametrize("keyed", [False, True])
def test_edge_votes_assemble_kernel(throughput_engine, keyed):
    """assemble_votes_kernel + the throughput kernels (generic prep/prep_r/main, keyed prep/main/finish)."""
    _check(throughput_engine, keyed)


@pytest.mark.parametrize("lens", [(1024, 4096), (3000, 3001)])
def test_generic_batch_long_messages(generic_engine, lens):
    """tmed_verify_batch with 1-4 KB messages (the ABI takes any length; the SHA-512 block loop is
    per lane: 17-65 blocks here, mixed in one wave), valid and with one flipped message bit."""
    rng = np.random.default_rng(lens[0])
    n = 300
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ml = rng.integers(lens[0], lens[1] + 1, n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(ml)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = generic_engine.sign_arrays(seeds, msgs, offs.astype(np.uint32))
    for i in range(0, n, 5):  # a flipped bit inside each 5th message (after signing)
        msgs[int(offs[i]) + int(rng.integers(0, int(ml[i])))] ^= 0x08
    out = generic_engine.verify_arrays(pubs, sigs, msgs, offs.astype(np.uint32))
    exp = port.verify_batch(pubs, sigs, msgs, offs, 16)
    assert int((out != exp).sum()) == 0
    assert int(exp.sum()) == n - len(range(0, n, 5))
