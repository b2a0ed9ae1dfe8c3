"""Shared scenario generator for the commit-seam parity tests (test helper)."""
import random

from oracle import commit as C
from oracle.fixtures import make_block_id, make_commit, make_valset, resign, seed_of

import tmed.types as T


def to_product(vs: C.ValidatorSet, cm: C.Commit):
    pv = T.ValidatorSet([T.Validator(v.pub_key, v.voting_power, v.proposer_priority, v.address) for v in vs.validators])
    pc = T.Commit(cm.height, cm.round, T.BlockID(cm.block_id.hash, cm.block_id.psh_total, cm.block_id.psh_hash),
                  [T.CommitSig(s.flag, s.address, s.timestamp, s.signature) for s in cm.signatures])
    return pv, pc


def pbid(b: C.BlockID):
    return T.BlockID(b.hash, b.psh_total, b.psh_hash)


def scenarios(seed=1, count=60, chains=("test_chain_id", "Lalande21185", "")):
    """Yield (mode, oracle_vs, product_vs, chain, oracle_bid, height, oracle_commit, product_commit, num, den)."""
    rng = random.Random(seed)
    for k in range(count):
        n = rng.choice([1, 2, 3, 4, 7, 10, 31])
        powers = [rng.choice([1, 10, 10, 100]) for _ in range(n)]
        vs, seeds = make_valset([seed_of("sc%d" % k, i) for i in range(n)], powers)
        chain = rng.choice(list(chains))
        bid = make_block_id("sc%d" % k)
        h = rng.randrange(1, 10**6)
        flags = [rng.choice([C.FLAG_COMMIT] * 6 + [C.FLAG_NIL, C.FLAG_ABSENT]) for _ in range(n)]
        cm = make_commit(vs, seeds, chain, h, rng.randrange(3), bid, flags=flags)
        # corruptions
        for _ in range(rng.choice([0, 0, 1, 2])):
            i = rng.randrange(n)
            if cm.signatures[i].flag != C.FLAG_ABSENT:
                kind = rng.randrange(3)
                if kind == 0:
                    resign(cm, i, seeds[i], "other-chain")
                elif kind == 1 and cm.signatures[i].signature:
                    s = bytearray(cm.signatures[i].signature)
                    s[rng.randrange(len(s))] ^= 1
                    cm.signatures[i].signature = bytes(s)
                elif kind == 2:
                    cm.signatures[i].signature = cm.signatures[i].signature[:rng.randrange(64)]
        mode = rng.randrange(3)
        want_bid, want_h = bid, h
        r = rng.random()
        if r < 0.05:
            want_h = h + 1
        elif r < 0.1:
            want_bid = make_block_id("zz%d" % k)
        num, den = rng.choice([(1, 3), (2, 3), (1, 1), (1, 0)] if rng.random() < 0.1 else [(1, 3), (2, 3)])
        if mode == 2 and rng.random() < 0.3 and n > 2:
            # double vote: duplicate an address among ForBlock sigs
            fb = [i for i in range(n) if cm.signatures[i].flag == C.FLAG_COMMIT]
            if len(fb) >= 2:
                cm.signatures[fb[-1]].address = cm.signatures[fb[0]].address
        tvs = vs
        if mode == 2 and rng.random() < 0.3:
            other, _ = make_valset([seed_of("oth%d" % k, i) for i in range(2)], [5, 5])
            tvs = C.ValidatorSet(other.validators + vs.validators) if rng.random() < 0.5 else other
        pv, pc = to_product(tvs, cm)
        yield mode, tvs, pv, chain, want_bid, want_h, cm, pc, num, den


def oracle_result(mode, vs, chain, bid, h, cm, num, den):
    if mode == 0:
        return C.verify_commit(vs, chain, bid, h, cm)
    if mode == 1:
        return C.verify_commit_light(vs, chain, bid, h, cm)
    return C.verify_commit_light_trusting(vs, chain, cm, num, den)


def same(a, b):
    if a is None or b is None:
        return a is None and b is None
    return type(a).__name__ == type(b).__name__ and str(a) == str(b)
