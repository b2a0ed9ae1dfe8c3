"""Synthetic validator sets and commits for the oracle tests (TEST INFRASTRUCTURE ONLY).

Mirrors the reference's test generators: ``types.RandValidatorSet``
(types/validator_set.go:1027-1042; sorted by power desc then address asc,
:906-911), ``types.MakeCommit`` (types/test_util.go:12-38) and
``makeBlockIDRandom`` (types/block_test.go:175-183, PSH total 123) — with
seeded keys instead of crypto/rand so fixtures are reproducible.
"""
from __future__ import annotations

import hashlib

from . import ed25519_go as E
from . import port
from .commit import FLAG_ABSENT, FLAG_COMMIT, FLAG_NIL, BlockID, Commit, CommitSig, Validator, ValidatorSet


def seed_of(tag: str, i: int) -> bytes:
    return hashlib.sha256(("%s-%d" % (tag, i)).encode()).digest()


def make_block_id(tag: str = "block") -> BlockID:
    return BlockID(hashlib.sha256(tag.encode()).digest(), 123, hashlib.sha256((tag + "/psh").encode()).digest())


def make_valset(seeds, powers, fast=True):
    pubs = [port.pubkey_from_seed(s) if fast else E.pubkey_from_seed(s) for s in seeds]
    vals = [(Validator(p, pw), s) for p, pw, s in zip(pubs, powers, seeds)]
    vals.sort(key=lambda vs: (-vs[0].voting_power, vs[0].address))
    return ValidatorSet([v for v, _ in vals]), [s for _, s in vals]


def make_commit(vs: ValidatorSet, seeds, chain_id: str, height: int, round_: int, block_id: BlockID,
                ts_base=(1672531200, 0), flags=None, fast=True) -> Commit:
    sigs = []
    commit = Commit(height, round_, block_id, sigs)
    for i, v in enumerate(vs.validators):
        f = FLAG_COMMIT if flags is None else flags[i]
        if f == FLAG_ABSENT:
            sigs.append(CommitSig(FLAG_ABSENT))
            continue
        ts = (ts_base[0] + i // 1000, ts_base[1] + (i % 1000) * 1_000_000)
        sigs.append(CommitSig(f, v.address, ts, b""))
        msg = commit.vote_sign_bytes(chain_id, i)
        sigs[-1].signature = port.sign(seeds[i], msg) if fast else E.sign(seeds[i], msg)
    return commit


def resign(commit: Commit, idx: int, seed: bytes, chain_id: str):
    """Replace signature #idx by a signature over the vote for another chain ID (malleation)."""
    msg = commit.vote_sign_bytes(chain_id, idx)
    commit.signatures[idx].signature = port.sign(seed, msg)
