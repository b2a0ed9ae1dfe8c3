"""Commit-verification loops restated on the CPU (TEST INFRASTRUCTURE ONLY).

Line-by-line restatement of ``types/validator_set.go``:
* ``VerifyCommit``               :667-714
* ``VerifyCommitLight``          :722-765
* ``VerifyCommitLightTrusting``  :775-826
* ``GetByAddress``               :270-278 (O(n) scan, first match)
* ``TotalVotingPower``           :298-321
* ``ErrNotEnoughVotingPowerSigned`` :856-863, ``safeMul`` :1086-1105
* ``types/errors.go:21-41``  ErrInvalidCommitHeight / ErrInvalidCommitSignatures
* ``types/block.go:577-634``  BlockIDFlag, ForBlock, Absent; ``:652-665`` CommitSig.BlockID

Errors are returned (Go style), never raised; ``str(err)`` is the Go ``err.Error()`` text.
The per-signature primitive is injectable (``verify_fn``) so that tests can
replay the loops over a bit vector the way the GPU seam does.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Callable, List, Optional

from . import ed25519_go
from .signbytes import PRECOMMIT_TYPE, vote_sign_bytes

FLAG_ABSENT = 1
FLAG_COMMIT = 2
FLAG_NIL = 3

MAX_INT64 = (1 << 63) - 1
MAX_TOTAL_VOTING_POWER = MAX_INT64 // 8


def _hexu(b: bytes) -> str:
    return b.hex().upper()


def fingerprint(b: bytes) -> bytes:
    return (bytes(b[:6]) + b"\x00" * 6)[:6]


@dataclass
class BlockID:
    hash: bytes = b""
    psh_total: int = 0
    psh_hash: bytes = b""

    def equals(self, o: "BlockID") -> bool:
        return self.hash == o.hash and self.psh_total == o.psh_total and self.psh_hash == o.psh_hash

    def is_zero(self) -> bool:
        return len(self.hash) == 0 and self.psh_total == 0 and len(self.psh_hash) == 0

    def __str__(self) -> str:  # types/block.go:1217-1219, part_set.go:103-105
        return "%s:%d:%s" % (_hexu(self.hash), self.psh_total, _hexu(fingerprint(self.psh_hash)))

    def as_tuple(self):
        return (self.hash, self.psh_total, self.psh_hash)


@dataclass
class CommitSig:
    flag: int
    address: bytes = b""
    timestamp: tuple = (-62135596800, 0)
    signature: bytes = b""

    def for_block(self) -> bool:
        return self.flag == FLAG_COMMIT

    def absent(self) -> bool:
        return self.flag == FLAG_ABSENT

    def block_id(self, commit_block_id: BlockID) -> BlockID:
        if self.flag in (FLAG_ABSENT, FLAG_NIL):
            return BlockID()
        if self.flag == FLAG_COMMIT:
            return commit_block_id
        raise RuntimeError("Unknown BlockIDFlag: %d" % self.flag)  # block.go:663 panics


@dataclass
class Commit:
    height: int
    round: int
    block_id: BlockID
    signatures: List[CommitSig]

    def vote_sign_bytes(self, chain_id: str, idx: int) -> bytes:
        """``Commit.VoteSignBytes`` (types/block.go:807-810)."""
        cs = self.signatures[idx]
        bid = cs.block_id(self.block_id)
        return vote_sign_bytes(chain_id, PRECOMMIT_TYPE, self.height, self.round,
                               bid.as_tuple(), cs.timestamp)


def address_of(pub: bytes) -> bytes:
    """``PubKey.Address`` = SHA-256(pub)[:20] (crypto/ed25519/ed25519.go:136-141)."""
    return hashlib.sha256(pub).digest()[:20]


@dataclass
class Validator:
    pub_key: bytes
    voting_power: int
    proposer_priority: int = 0
    address: bytes = b""

    def __post_init__(self):
        if not self.address:
            self.address = address_of(self.pub_key)

    def __str__(self) -> str:  # types/validator.go:92-101
        return "Validator{%s PubKeyEd25519{%s} VP:%d A:%d}" % (
            _hexu(self.address), _hexu(self.pub_key), self.voting_power, self.proposer_priority)


@dataclass
class ValidatorSet:
    validators: List[Validator]
    _total: int = field(default=0, repr=False)

    def size(self) -> int:
        return len(self.validators)

    def total_voting_power(self) -> int:
        if self._total == 0:
            s = 0
            for v in self.validators:
                s = min(s + v.voting_power, MAX_INT64)  # safeAddClip
                if s > MAX_TOTAL_VOTING_POWER:
                    raise RuntimeError("Total voting power should be guarded to not exceed %d; got: %d"
                                       % (MAX_TOTAL_VOTING_POWER, s))
            self._total = s
        return self._total

    def get_by_address(self, addr: bytes):
        for i, v in enumerate(self.validators):
            if v.address == addr:
                return i, v
        return -1, None


# ---------------------------------------------------------------------------
# Errors (Go error values).

class GoError:
    def __init__(self, msg: str):
        self.msg = msg

    def __str__(self):
        return self.msg

    def __eq__(self, o):
        return type(self) is type(o) and str(self) == str(o)

    def __repr__(self):
        return "%s(%r)" % (type(self).__name__, self.msg)


class ErrInvalidCommitSignatures(GoError):
    def __init__(self, expected: int, actual: int):
        self.expected, self.actual = expected, actual
        super().__init__("Invalid commit -- wrong set size: %d vs %d" % (expected, actual))


class ErrInvalidCommitHeight(GoError):
    def __init__(self, expected: int, actual: int):
        self.expected, self.actual = expected, actual
        super().__init__("Invalid commit -- wrong height: %d vs %d" % (expected, actual))


class ErrNotEnoughVotingPowerSigned(GoError):
    def __init__(self, got: int, needed: int):
        self.got, self.needed = got, needed
        super().__init__("invalid commit -- insufficient voting power: got %d, needed more than %d"
                         % (got, needed))


def _go_div(a: int, b: int) -> int:
    """int64 division truncating toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _wrap64(x: int) -> int:
    """int64 two's-complement wrap (Go's arithmetic on int64)."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def safe_mul(a: int, b: int):
    """types/validator_set.go:1086-1105, with Go's wrapping: -MinInt64 == MinInt64, so for
    b = MinInt64 (int64(Numerator) of 2^63) |b| stays negative and MaxInt64 / |b| truncates to 0."""
    if a == 0 or b == 0:
        return 0, False
    abs_b = _wrap64(-b) if b < 0 else b
    abs_a = _wrap64(-a) if a < 0 else a
    if abs_a > _go_div(MAX_INT64, abs_b):
        return 0, True
    return _wrap64(a * b), False


def _default_verify(pub, msg, sig):
    return ed25519_go.verify(pub, msg, sig)


VerifyFn = Callable[[bytes, bytes, bytes], bool]


def _prechecks(vals: ValidatorSet, block_id: BlockID, height: int, commit: Commit) -> Optional[GoError]:
    if vals.size() != len(commit.signatures):
        return ErrInvalidCommitSignatures(vals.size(), len(commit.signatures))
    if height != commit.height:
        return ErrInvalidCommitHeight(height, commit.height)
    if not block_id.equals(commit.block_id):
        return GoError("invalid commit -- wrong block ID: want %s, got %s" % (block_id, commit.block_id))
    return None


def verify_commit(vals, chain_id, block_id, height, commit, verify_fn: VerifyFn = _default_verify):
    """``ValidatorSet.VerifyCommit`` (types/validator_set.go:667-714)."""
    err = _prechecks(vals, block_id, height, commit)
    if err is not None:
        return err
    tallied = 0
    needed = _go_div(vals.total_voting_power() * 2, 3)
    for idx, cs in enumerate(commit.signatures):
        if cs.absent():
            continue
        val = vals.validators[idx]
        msg = commit.vote_sign_bytes(chain_id, idx)
        if not verify_fn(val.pub_key, msg, cs.signature):
            return GoError("wrong signature (#%d): %s" % (idx, _hexu(cs.signature)))
        if cs.for_block():
            tallied += val.voting_power
    if tallied <= needed:
        return ErrNotEnoughVotingPowerSigned(tallied, needed)
    return None


def verify_commit_light(vals, chain_id, block_id, height, commit, verify_fn: VerifyFn = _default_verify):
    """``ValidatorSet.VerifyCommitLight`` (types/validator_set.go:722-765)."""
    err = _prechecks(vals, block_id, height, commit)
    if err is not None:
        return err
    tallied = 0
    needed = _go_div(vals.total_voting_power() * 2, 3)
    for idx, cs in enumerate(commit.signatures):
        if not cs.for_block():
            continue
        val = vals.validators[idx]
        msg = commit.vote_sign_bytes(chain_id, idx)
        if not verify_fn(val.pub_key, msg, cs.signature):
            return GoError("wrong signature (#%d): %s" % (idx, _hexu(cs.signature)))
        tallied += val.voting_power
        if tallied > needed:
            return None
    return ErrNotEnoughVotingPowerSigned(tallied, needed)


def verify_commit_light_trusting(vals, chain_id, commit, trust_num: int, trust_den: int,
                                 verify_fn: VerifyFn = _default_verify):
    """``ValidatorSet.VerifyCommitLightTrusting`` (types/validator_set.go:775-826)."""
    if trust_den == 0:
        return GoError("trustLevel has zero Denominator")
    tallied = 0
    seen = {}
    prod, overflow = safe_mul(vals.total_voting_power(), trust_num)
    if overflow:
        return GoError("int64 overflow while calculating voting power needed. "
                       "please provide smaller trustLevel numerator")
    needed = _go_div(prod, trust_den)
    for idx, cs in enumerate(commit.signatures):
        if not cs.for_block():
            continue
        val_idx, val = vals.get_by_address(cs.address)
        if val is not None:
            if val_idx in seen:
                return GoError("double vote from %s (%d and %d)" % (val, seen[val_idx], idx))
            seen[val_idx] = idx
            msg = commit.vote_sign_bytes(chain_id, idx)
            if not verify_fn(val.pub_key, msg, cs.signature):
                return GoError("wrong signature (#%d): %s" % (idx, _hexu(cs.signature)))
            tallied += val.voting_power
            if tallied > needed:
                return None
    return ErrNotEnoughVotingPowerSigned(tallied, needed)
