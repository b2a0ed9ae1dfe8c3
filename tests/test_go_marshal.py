"""The Go shim's host marshal in compiled code (tendermint-fork_amd/shim/go_marshal.cpp): commits and
validator sets laid out as Go holds them (types/block.go:595-600, 737-752; types/validator_set.go:
51-58) flattened into the C ABI structs, then through the seam with the oracle as the batch
verifier (tmed_verify_commits_with: CPU only) — every outcome equal to the oracle's restatement of
the reference loops.  The blocksync flatten stops each Light commit at its 2/3 crossing (the loop
never reads further): windows with bad signatures before / after the crossing, nil and absent votes,
short signatures, a wrong set size and a commit that never crosses check that this is exact."""
import numpy as np

from commit_cases import edge_scenarios, oracle_outcome, pbid, same_outcome, scenarios
from oracle import commit as C
from oracle import port
from oracle.fixtures import make_block_id, make_commit, make_valset, seed_of
import tmed.types as T
from tmed import gomarshal as G


def oracle_verifier(pubs, sigs, lens, msgs, offs):
    out = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 4)
    out[lens != 64] = 0
    return out


def _errors(res, reqs):
    return [T._to_error(res[q].code, res[q], reqs[q][1], reqs[q][3], reqs[q][5]) for q in range(len(reqs))]


def test_requests_marshal_matches_reference_loops():
    """Random and edge corpora (every mode; Trusting sets that differ from the commit's, duplicate
    addresses, 0/19/21-byte addresses, unknown flags, malformed BlockID hashes) marshalled from Go
    layouts by the compiled shim; one C valset / commit per distinct object; set hashes passed."""
    heap = G.GoHeap()
    reqs, exp, rows = [], [], []
    sets, commits = {}, {}
    cases = list(scenarios(seed=31, count=60)) + list(edge_scenarios(seed=32, count=30))
    for k, (mode, vs, pv, chain, bid, h, cm, pc, num, den) in enumerate(cases):
        if chain != "test_chain_id":
            continue  # one chain ID per marshalled call (as one light client / one chain)
        si = sets.setdefault(id(pv), heap.valset(pv))
        ci = commits.setdefault(id(pc), heap.commit(G.packed_of(pc)))
        if mode != T.MODE_LIGHT_TRUSTING and bytes(pc.block_id.hash) != bytes(bid.hash):
            continue  # the marshal's expected BlockID is the commit's own (the bench's shape)
        if mode != T.MODE_LIGHT_TRUSTING and (pc.block_id.psh_total, bytes(pc.block_id.psh_hash)) != \
                (bid.psh_total, bytes(bid.psh_hash)):
            continue
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
        exp.append(oracle_outcome(mode, vs, chain, bid, h, cm, num, den))
        rows.append((mode, si, ci, h, num, den))
    assert len(reqs) > 30
    a = np.array(rows, np.int64)
    hashes = np.random.default_rng(1).integers(0, 256, (len(sets), 32), dtype=np.uint8)
    m = G.Marshal(threads=4)
    for forget in (True, False):  # fresh set flattening, then the shim's per-set cache
        rq = m.requests(heap, a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4], a[:, 5], "test_chain_id",
                        set_hashes=hashes, forget_sets=forget)
        res = T.run_requests(None, rq, len(reqs), verifier=oracle_verifier)
        got = _errors(res, reqs)
        bad = [(q, got[q], exp[q]) for q in range(len(reqs)) if not same_outcome(got[q], exp[q])]
        assert not bad, bad[:4]
        sh = rq[0].vals.contents.set_hash  # each set's ValidatorsHash reaches the seam as set_hash
        assert np.ctypeslib.as_array(ctypes_u8(sh), (32,)).tobytes() == hashes[int(a[0, 1])].tobytes()
    assert sum(e is not None for e in exp) > 5
    m.free()
    heap.free()


def ctypes_u8(p):
    import ctypes
    return ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8))


def test_window_marshal_stops_at_the_light_crossing():
    vs, seeds = make_valset([seed_of("gmw", i) for i in range(40)], [1 + (i % 7) * 5 for i in range(40)])
    pv = T.ValidatorSet([T.Validator(v.pub_key, v.voting_power, v.proposer_priority, v.address) for v in vs.validators])
    heap = G.GoHeap()
    si = heap.valset(pv)
    blocks, exp = [], []
    total = sum(v.voting_power for v in vs.validators)
    for b in range(14):
        bid = make_block_id("gmw%d" % b)
        flags = [C.FLAG_COMMIT] * 40
        if b % 3 == 1:
            flags[2] = C.FLAG_NIL
            flags[5] = C.FLAG_ABSENT
        if b == 9:  # too few votes for block: never crosses -> ErrNotEnoughVotingPowerSigned
            flags = [C.FLAG_NIL] * 26 + [C.FLAG_COMMIT] * 14
        cm = make_commit(vs, seeds, "test_chain_id", 100 + b, 0, bid, flags=flags)
        # where the Light loop stops
        tally, cross = 0, 40
        for i, cs in enumerate(cm.signatures):
            if cs.flag == C.FLAG_COMMIT:
                tally += vs.validators[i].voting_power
                if tally > total * 2 // 3:
                    cross = i
                    break
        if b % 4 == 2 and cross > 1:
            s = bytearray(cm.signatures[cross - 1].signature)  # before the crossing: wrong signature
            s[3] ^= 1
            cm.signatures[cross - 1].signature = bytes(s)
        if b % 4 == 3 and cross + 1 < 40:
            s = bytearray(cm.signatures[cross + 1].signature)  # after it: never read
            s[3] ^= 1
            cm.signatures[cross + 1].signature = bytes(s)
            cm.signatures[cross + 2].signature = b""         # nor this short one
        if b == 5 and cross > 0:
            cm.signatures[cross].signature = cm.signatures[cross].signature[:63]  # the crossing one: short
        pc = T.Commit(cm.height, cm.round, T.BlockID(bid.hash, bid.psh_total, bid.psh_hash),
                      [T.CommitSig(s.flag, s.address, s.timestamp, s.signature) for s in cm.signatures])
        if b == 12:  # a wrong set size: the size check fails before any signature
            pc.signatures = pc.signatures[:39]
            cm = C.Commit(cm.height, cm.round, cm.block_id, cm.signatures[:39])
        blocks.append(heap.commit(G.packed_of(pc)))
        exp.append(C.verify_commit_light(vs, "test_chain_id", bid, 100 + b, cm))
    m = G.Marshal(threads=3)
    arena = np.zeros(64 * 40 * len(blocks), np.uint8)
    w = m.window(heap, si, np.array(blocks), np.arange(100, 114), "test_chain_id",
                 set_hash=bytes(range(32)), sig_arena=arena.ctypes.data)
    win = w.contents
    assert win.n_blocks == 14 and win.vals.contents.addresses is None  # Light needs no addresses
    import ctypes
    reqs = (T._RequestC * 14)()
    cid = b"test_chain_id"
    hts = ctypes.cast(win.heights, ctypes.POINTER(ctypes.c_int64))
    for h in range(14):  # the window as the seam sees it: one Light request per block
        reqs[h] = T._RequestC(T.MODE_LIGHT, cid, len(cid), win.vals, ctypes.pointer(win.block_ids[h]), hts[h],
                              ctypes.pointer(win.commits[h]), 0, 0)
    res = T.run_requests(None, reqs, 14, verifier=oracle_verifier)
    for h in range(14):
        e = exp[h]
        if e is None:
            assert res[h].code == 0, (h, res[h].code)
        elif isinstance(e, C.ErrNotEnoughVotingPowerSigned):
            assert res[h].code == 5 and (res[h].got, res[h].needed) == (e.got, e.needed), h
        elif isinstance(e, C.ErrInvalidCommitSignatures):
            assert res[h].code == 1, h
        else:
            assert res[h].code == 4 and str(e).startswith("wrong signature (#%d)" % res[h].idx), (h, res[h].code, e)
    # the tail past each crossing was not marshalled: its flags read Absent, its signatures zero
    c0 = win.commits[0]
    flags = np.ctypeslib.as_array(ctypes_u8(c0.flags), (40,))
    assert (flags == 1).sum() > 0 and flags[0] == 2
    assert sum(e is None for e in exp) >= 5 and any(isinstance(e, C.ErrNotEnoughVotingPowerSigned) for e in exp)
    m.free()
    heap.free()
