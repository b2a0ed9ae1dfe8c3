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
            r2 = rng.random()
            if r2 < 0.35:
                tvs = C.ValidatorSet(other.validators + vs.validators)
            elif r2 < 0.7 or n <= 2:
                tvs = other
            else:  # validator 2's address also at position 0: signature 2 matches its own
                # position, but GetByAddress returns the first match (index 0)
                tvs = C.ValidatorSet([vs.validators[2]] + vs.validators[1:])
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


def oracle_outcome(mode, vs, chain, bid, h, cm, num, den):
    """oracle_result, or ("panic", idx) where the reference loop panics (unknown BlockIDFlag in
    CommitSig.BlockID, types/block.go:652-665; malformed hash in CanonicalizeBlockID,
    types/canonical.go:18-22) — idx = the signature whose sign-bytes it was building."""
    last = []
    orig = cm.vote_sign_bytes

    def vsb(chain_id, idx):
        last.append(idx)
        return orig(chain_id, idx)

    cm.vote_sign_bytes = vsb
    try:
        return oracle_result(mode, vs, chain, bid, h, cm, num, den)
    except (RuntimeError, ValueError):
        return ("panic", last[-1])
    finally:
        del cm.vote_sign_bytes


def same_outcome(got, exp):
    if isinstance(exp, tuple):
        return isinstance(got, T.GoPanic) and got.idx == exp[1]
    return not isinstance(got, T.GoPanic) and same(got, exp)


_Z00 = []


def address_ending_in_zero():
    """(seed, validator) whose address ends in 0x00: its 19-byte prefix zero-padded to 20 bytes
    equals the address, which a fixed 20-byte slot would wrongly match (GetByAddress uses
    bytes.Equal, types/validator_set.go:270-277)."""
    if not _Z00:
        from oracle import port
        for i in range(100000):
            s = seed_of("z00", i)
            p = port.pubkey_from_seed(s)
            if C.address_of(p)[19] == 0:
                _Z00.append((s, p))
                break
    return _Z00[0]


def edge_scenarios(seed=7, count=40, chains=("test_chain_id", "")):
    """Scenarios on which the reference loop panics or GetByAddress sees odd-length addresses:
    unknown BlockIDFlags (0, 4, 9, 255) in any mode, malformed BlockID hashes (31/33 bytes, the
    request's expected BlockID equal to the commit's so the prechecks pass), and ValidatorAddress
    lengths 0, 19 and 21 — including the 19-byte prefix of a real address that ends in 0x00.
    Yields the same tuples as scenarios()."""
    rng = random.Random(seed)
    zs, zp = address_ending_in_zero()
    for k in range(count):
        n = rng.choice([3, 4, 7, 10])
        seeds_in = [seed_of("ed%d" % k, i) for i in range(n - 1)] + [zs]
        vs, seeds = make_valset(seeds_in, [10] * n)
        chain = rng.choice(list(chains))
        bid = make_block_id("ed%d" % k)
        h = rng.randrange(1, 10**6)
        flags = [rng.choice([C.FLAG_COMMIT] * 5 + [C.FLAG_NIL, C.FLAG_ABSENT]) for _ in range(n)]
        cm = make_commit(vs, seeds, chain, h, rng.randrange(2), bid, flags=flags)
        if rng.random() < 0.4:  # one bad signature somewhere (before or after the odd input)
            i = rng.randrange(n)
            if cm.signatures[i].signature:
                s = bytearray(cm.signatures[i].signature)
                s[5] ^= 4
                cm.signatures[i].signature = bytes(s)
        kind = k % 3
        want_bid = bid
        if kind == 0:
            cm.signatures[rng.randrange(n)].flag = rng.choice([0, 4, 9, 255])
        elif kind == 1:
            if rng.random() < 0.5:
                cm.block_id = C.BlockID(bid.hash[:31], bid.psh_total, bid.psh_hash)
            else:
                cm.block_id = C.BlockID(bid.hash, bid.psh_total, bid.psh_hash + b"\x01")
            want_bid = cm.block_id
        else:
            zi = next(i for i, v in enumerate(vs.validators) if v.pub_key == zp)
            for i in rng.sample(range(n), min(n, 2)):
                if cm.signatures[i].flag == C.FLAG_ABSENT:
                    continue
                a = cm.signatures[i].address
                cm.signatures[i].address = rng.choice([b"", a[:19], a + b"\x00"])
            if cm.signatures[zi].flag != C.FLAG_ABSENT:
                cm.signatures[zi].address = vs.validators[zi].address[:19]
        mode = rng.randrange(3)
        pv, pc = to_product(vs, cm)
        yield mode, vs, pv, chain, want_bid, h, cm, pc, 1, 3
