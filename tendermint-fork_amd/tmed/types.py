"""Host mirror of the reference's commit types and the VerifyCommit* seam.

Python mirror of ``types.ValidatorSet.VerifyCommit``, ``VerifyCommitLight`` and
``VerifyCommitLightTrusting`` (reference ``types/validator_set.go:667-826``)
over the C ABI ``tmed_verify_commits`` (C++ plan/replay in
``csrc/commit.hip``): same argument meaning, same return convention (``None``
or an error value whose ``str()`` is Go's ``err.Error()``), same error types
(``ErrInvalidCommitSignatures``, ``ErrInvalidCommitHeight``,
``ErrNotEnoughVotingPowerSigned`` are what ``light/verifier.go:60-61`` and
``light/client.go:746`` type-switch on).  Batches of commits go to the GPU in
one launch via :func:`verify_commits`.
"""
from __future__ import annotations

import ctypes
import hashlib
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from ._native import TMED_OK, TmedError, lib

FLAG_ABSENT, FLAG_COMMIT, FLAG_NIL = 1, 2, 3        # types/block.go:577-584
MODE_COMMIT, MODE_LIGHT, MODE_LIGHT_TRUSTING = 0, 1, 2
MAX_INT64 = (1 << 63) - 1
MAX_TOTAL_VOTING_POWER = MAX_INT64 // 8            # types/validator_set.go:25
ZERO_TIME = (-62135596800, 0)


def _hexu(b: bytes) -> str:
    return bytes(b).hex().upper()


def address_of(pub: bytes) -> bytes:
    """ed25519 PubKey.Address = SHA-256(pub)[:20] (crypto/ed25519/ed25519.go:136-141)."""
    return hashlib.sha256(pub).digest()[:20]


# --------------------------------------------------------------------------- types

@dataclass
class BlockID:
    hash: bytes = b""
    psh_total: int = 0
    psh_hash: bytes = b""

    def equals(self, o: "BlockID") -> bool:
        return self.hash == o.hash and self.psh_total == o.psh_total and self.psh_hash == o.psh_hash

    def __str__(self):  # types/block.go:1217-1219 (+ PartSetHeader.String, part_set.go:103-105)
        return "%s:%d:%s" % (_hexu(self.hash), self.psh_total, _hexu((bytes(self.psh_hash[:6]) + bytes(6))[:6]))


@dataclass
class CommitSig:
    flag: int
    address: bytes = b""
    timestamp: tuple = ZERO_TIME
    signature: bytes = b""


@dataclass
class Commit:
    height: int
    round: int
    block_id: BlockID
    signatures: List[CommitSig]


@dataclass
class PackedCommit:
    """A Commit held as arrays (bulk workloads: blocksync replay, light-client batches)."""
    height: int
    round: int
    block_id: BlockID
    flags: np.ndarray        # u8[n]  BlockIDFlag
    addresses: np.ndarray    # u8[n,20]
    ts_seconds: np.ndarray   # i64[n]
    ts_nanos: np.ndarray     # i32[n]
    sigs: np.ndarray         # u8[n,64]
    sig_lens: np.ndarray     # u32[n]
    address_lens: Optional[np.ndarray] = None  # u32[n] len(ValidatorAddress); None = all 20

    @property
    def signatures(self):
        return _PackedSigs(self)


class _PackedSigs:
    def __init__(self, pc):
        self.pc = pc

    def __len__(self):
        return self.pc.flags.shape[0]

    def __getitem__(self, i):
        pc = self.pc
        al = 20 if pc.address_lens is None else int(pc.address_lens[i])
        addr = pc.addresses[i].tobytes() if al == 20 else bytes(al)  # other lengths: content never compared
        return CommitSig(int(pc.flags[i]), addr, (int(pc.ts_seconds[i]), int(pc.ts_nanos[i])),
                         pc.sigs[i, :int(pc.sig_lens[i])].tobytes())


@dataclass
class Validator:
    pub_key: bytes
    voting_power: int
    proposer_priority: int = 0
    address: bytes = b""

    def __post_init__(self):
        if not self.address:
            self.address = address_of(self.pub_key)

    def __str__(self):  # types/validator.go:92-101
        return "Validator{%s PubKeyEd25519{%s} VP:%d A:%d}" % (
            _hexu(self.address), _hexu(self.pub_key), self.voting_power, self.proposer_priority)


@dataclass
class ValidatorSet:
    validators: List[Validator]
    _total: int = field(default=0, repr=False)
    _packed: Optional[tuple] = field(default=None, repr=False)
    keyset: int = field(default=0, repr=False)                       # tmed_keyset_load handle (0: the key-set cache)
    keyset_index: Optional[np.ndarray] = field(default=None, repr=False)  # validator -> key-set index (u32)
    set_hash: Optional[bytes] = field(default=None, repr=False)      # ValidatorSet.Hash() (key-set cache key)

    def size(self) -> int:
        return len(self.validators)

    def total_voting_power(self) -> int:  # types/validator_set.go:298-321
        if self._total == 0:
            s = 0
            for v in self.validators:
                s = min(s + v.voting_power, MAX_INT64)
                if s > MAX_TOTAL_VOTING_POWER:
                    raise RuntimeError("Total voting power should be guarded to not exceed %d; got: %d"
                                       % (MAX_TOTAL_VOTING_POWER, s))
            self._total = s
        return self._total

    def packed(self):
        if self._packed is None:
            n = len(self.validators)
            pubs = np.zeros((max(n, 1), 32), np.uint8)
            addrs = np.zeros((max(n, 1), 20), np.uint8)
            for i, v in enumerate(self.validators):
                if len(v.pub_key) != 32:
                    raise ValueError("not an ed25519 key: the reference path handles it")
                pubs[i] = np.frombuffer(v.pub_key, np.uint8)
                addrs[i] = np.frombuffer(v.address, np.uint8)
            powers = np.array([v.voting_power for v in self.validators] or [0], np.int64)
            self._packed = (pubs, powers, addrs)
        return self._packed

    # reference method names
    def verify_commit(self, engine, chain_id: str, block_id: BlockID, height: int, commit: Commit):
        return _raise_panic(verify_commits(engine, [(MODE_COMMIT, self, chain_id, block_id, height, commit, 0, 0)])[0])

    def verify_commit_light(self, engine, chain_id: str, block_id: BlockID, height: int, commit: Commit):
        return _raise_panic(verify_commits(engine, [(MODE_LIGHT, self, chain_id, block_id, height, commit, 0, 0)])[0])

    def verify_commit_light_trusting(self, engine, chain_id: str, commit: Commit, num: int, den: int):
        return _raise_panic(verify_commits(engine, [(MODE_LIGHT_TRUSTING, self, chain_id, None, 0, commit, num, den)])[0])


def _raise_panic(res):
    if isinstance(res, GoPanic):
        raise res
    return res


# --------------------------------------------------------------------------- errors

class GoError:
    def __init__(self, msg: str):
        self.msg = msg

    def __str__(self):
        return self.msg

    def __repr__(self):
        return "%s(%r)" % (type(self).__name__, self.msg)

    def __eq__(self, o):
        return type(self).__name__ == type(o).__name__ and str(self) == str(o)


class ErrInvalidCommitSignatures(GoError):  # types/errors.go:32-41
    def __init__(self, expected, actual):
        self.expected, self.actual = expected, actual
        super().__init__("Invalid commit -- wrong set size: %d vs %d" % (expected, actual))


class ErrInvalidCommitHeight(GoError):  # types/errors.go:21-30
    def __init__(self, expected, actual):
        self.expected, self.actual = expected, actual
        super().__init__("Invalid commit -- wrong height: %d vs %d" % (expected, actual))


class ErrNotEnoughVotingPowerSigned(GoError):  # types/validator_set.go:856-863
    def __init__(self, got, needed):
        self.got, self.needed = got, needed
        super().__init__("invalid commit -- insufficient voting power: got %d, needed more than %d" % (got, needed))


class GoPanic(RuntimeError):
    """The reference loop panics at signature ``idx`` (TMED_COMMIT_PANIC): an unknown BlockIDFlag in
    VerifyCommit (types/block.go:652-665) or a malformed BlockID hash reaching CanonicalizeBlockID
    (types/canonical.go:18-22).  The reference-named methods raise it, like Go's panic; the batch
    functions return it in that request's slot."""

    def __init__(self, idx):
        self.idx = idx
        super().__init__("reference panics at signature #%d" % idx)


# --------------------------------------------------------------------------- ABI structs

class _BlockIDC(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_void_p), ("hash_len", ctypes.c_uint32), ("psh_total", ctypes.c_uint32),
                ("psh_hash", ctypes.c_void_p), ("psh_hash_len", ctypes.c_uint32)]


class _ValsetC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("pubkeys", ctypes.c_void_p), ("powers", ctypes.c_void_p),
                ("addresses", ctypes.c_void_p), ("total_power", ctypes.c_int64), ("keyset", ctypes.c_uint64),
                ("keyset_index", ctypes.c_void_p), ("set_hash", ctypes.c_void_p)]


class _CommitC(ctypes.Structure):
    _fields_ = [("height", ctypes.c_int64), ("round", ctypes.c_int32), ("block_id", _BlockIDC),
                ("n_sigs", ctypes.c_size_t), ("flags", ctypes.c_void_p), ("addresses", ctypes.c_void_p),
                ("ts_seconds", ctypes.c_void_p), ("ts_nanos", ctypes.c_void_p), ("sigs", ctypes.c_void_p),
                ("sig_lens", ctypes.c_void_p), ("address_lens", ctypes.c_void_p)]


class _RequestC(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("chain_id", ctypes.c_char_p), ("chain_id_len", ctypes.c_uint32),
                ("vals", ctypes.POINTER(_ValsetC)), ("block_id", ctypes.POINTER(_BlockIDC)),
                ("height", ctypes.c_int64), ("commit", ctypes.POINTER(_CommitC)),
                ("trust_num", ctypes.c_int64), ("trust_den", ctypes.c_int64)]


class _ResultC(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int), ("got", ctypes.c_int64), ("needed", ctypes.c_int64),
                ("expected", ctypes.c_int64), ("actual", ctypes.c_int64), ("idx", ctypes.c_int32),
                ("idx_first", ctypes.c_int32), ("val_idx", ctypes.c_int32), ("verified", ctypes.c_uint32)]


class _BlocksyncWindowC(ctypes.Structure):
    _fields_ = [("chain_id", ctypes.c_char_p), ("chain_id_len", ctypes.c_uint32), ("vals", ctypes.POINTER(_ValsetC)),
                ("n_blocks", ctypes.c_size_t), ("block_ids", ctypes.POINTER(_BlockIDC)),
                ("heights", ctypes.c_void_p), ("commits", ctypes.POINTER(_CommitC))]


VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def _bind():
    l = lib()
    if l.tmed_verify_commits.argtypes is None:
        l.tmed_verify_commits.restype = ctypes.c_int
        l.tmed_verify_commits.argtypes = [ctypes.c_void_p, ctypes.POINTER(_RequestC), ctypes.c_size_t,
                                          ctypes.POINTER(_ResultC)]
        l.tmed_blocksync_verify.restype = ctypes.c_int
        l.tmed_blocksync_verify.argtypes = [ctypes.c_void_p, ctypes.POINTER(_BlocksyncWindowC), ctypes.c_uint32,
                                            ctypes.POINTER(_ResultC)]
        l.tmed_blocksync_submit.restype = ctypes.c_int
        l.tmed_blocksync_submit.argtypes = l.tmed_blocksync_verify.argtypes
        l.tmed_blocksync_wait.restype = ctypes.c_int
        l.tmed_blocksync_wait.argtypes = [ctypes.c_void_p]
        l.tmed_verify_commits_with.restype = ctypes.c_int
        l.tmed_verify_commits_with.argtypes = [ctypes.POINTER(_RequestC), ctypes.c_size_t,
                                               ctypes.POINTER(_ResultC), VERIFY_FN, ctypes.c_void_p]
        l.tmed_verify_commits_multi.restype = ctypes.c_int
        l.tmed_verify_commits_multi.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                                ctypes.POINTER(_RequestC), ctypes.c_size_t, ctypes.POINTER(_ResultC)]
        l.tmed_blocksync_verify_multi.restype = ctypes.c_int
        l.tmed_blocksync_verify_multi.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                                  ctypes.POINTER(_BlocksyncWindowC), ctypes.c_uint32,
                                                  ctypes.POINTER(_ResultC)]
        l.tmed_seam_phase_us.restype = ctypes.c_int
        l.tmed_seam_phase_us.argtypes = [ctypes.POINTER(ctypes.c_double)]
    return l


def blocksync_wait(engine):
    """tmed_blocksync_wait: collect every window submitted on the engine (BlocksyncWindow.submit)."""
    rc = _bind().tmed_blocksync_wait(engine._h)
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_blocksync_wait")


def _ctx_array(engines):
    """ctypes array of the contexts of several engines (one per GPU, the same process)."""
    return (ctypes.c_void_p * len(engines))(*[e._h for e in engines])


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _block_id_c(b: BlockID, keep):
    h, ph = bytes(b.hash), bytes(b.psh_hash)
    keep.extend([h, ph])
    return _BlockIDC(ctypes.cast(ctypes.c_char_p(h), ctypes.c_void_p), len(h), b.psh_total,
                     ctypes.cast(ctypes.c_char_p(ph), ctypes.c_void_p), len(ph))


def _commit_c(c, keep):
    if isinstance(c, PackedCommit):
        arrs = [np.ascontiguousarray(c.flags, np.uint8), np.ascontiguousarray(c.addresses, np.uint8),
                np.ascontiguousarray(c.ts_seconds, np.int64), np.ascontiguousarray(c.ts_nanos, np.int32),
                np.ascontiguousarray(c.sigs, np.uint8), np.ascontiguousarray(c.sig_lens, np.uint32)]
        al = None if c.address_lens is None else np.ascontiguousarray(c.address_lens, np.uint32)
        keep.extend(arrs + [al])
        return _CommitC(c.height, c.round, _block_id_c(c.block_id, keep), arrs[0].shape[0], *[_ptr(a) for a in arrs],
                        None if al is None else _ptr(al))
    n = len(c.signatures)
    m = max(n, 1)
    flags = np.zeros(m, np.uint8)
    addrs = np.zeros((m, 20), np.uint8)
    sec = np.zeros(m, np.int64)
    nan = np.zeros(m, np.int32)
    sigs = np.zeros((m, 64), np.uint8)
    lens = np.zeros(m, np.uint32)
    alens = np.zeros(m, np.uint32)
    for i, cs in enumerate(c.signatures):
        flags[i] = cs.flag
        alens[i] = len(cs.address)  # only a 20-byte address can equal a validator's (GetByAddress)
        if len(cs.address) == 20:
            addrs[i] = np.frombuffer(cs.address, np.uint8)
        sec[i], nan[i] = cs.timestamp
        s = cs.signature[:64]
        if s:
            sigs[i, :len(s)] = np.frombuffer(s, np.uint8)
        lens[i] = len(cs.signature)
    keep.extend([flags, addrs, sec, nan, sigs, lens, alens])
    return _CommitC(c.height, c.round, _block_id_c(c.block_id, keep), n, _ptr(flags), _ptr(addrs), _ptr(sec),
                    _ptr(nan), _ptr(sigs), _ptr(lens), _ptr(alens))


def _valset_c(vals: ValidatorSet, keep) -> _ValsetC:
    """tmed_valset of a ValidatorSet (its packed arrays, handle, key-set index and set_hash)."""
    pubs, powers, addrs = vals.packed()
    kidx = getattr(vals, "keyset_index", None)
    sh = getattr(vals, "set_hash", None)
    if sh is not None and len(sh) != 32:
        raise ValueError("set_hash must be ValidatorSet.Hash() (32 bytes)")
    sh = None if sh is None else bytes(sh)
    keep.extend([pubs, powers, addrs, kidx, sh])
    return _ValsetC(len(vals.validators), _ptr(pubs), _ptr(powers), _ptr(addrs), vals.total_voting_power(),
                    getattr(vals, "keyset", 0) or 0, None if kidx is None else _ptr(kidx),
                    None if sh is None else ctypes.cast(ctypes.c_char_p(sh), ctypes.c_void_p))


def _to_error(code, r: _ResultC, vals: ValidatorSet, block_id, commit: Commit):
    if code == 0:
        return None
    if code == 1:
        return ErrInvalidCommitSignatures(r.expected, r.actual)
    if code == 2:
        return ErrInvalidCommitHeight(r.expected, r.actual)
    if code == 3:
        return GoError("invalid commit -- wrong block ID: want %s, got %s" % (block_id, commit.block_id))
    if code == 4:
        return GoError("wrong signature (#%d): %s" % (r.idx, _hexu(commit.signatures[r.idx].signature)))
    if code == 5:
        return ErrNotEnoughVotingPowerSigned(r.got, r.needed)
    if code == 6:
        return GoError("double vote from %s (%d and %d)" % (vals.validators[r.val_idx], r.idx_first, r.idx))
    if code == 7:
        return GoError("trustLevel has zero Denominator")
    if code == 8:
        return GoError("int64 overflow while calculating voting power needed. please provide smaller trustLevel numerator")
    if code == 9:
        return GoPanic(r.idx)  # a batch reports it per request; the reference-named methods raise it
    raise RuntimeError("tmed: unknown commit outcome %d" % code)


class PreparedBatch:
    """Requests packed into C structs once, for repeated timing of the seam itself
    (host sign-bytes + staging + device + replay), without Python packing in the loop."""

    def __init__(self, requests: Sequence[tuple]):
        self.requests = list(requests)
        self.keep = []
        n = len(self.requests)
        self.n = n
        self.reqs = (_RequestC * max(n, 1))()
        vcs = {}  # one tmed_valset per ValidatorSet object (the seam resolves each set once)
        ccs = {}  # one tmed_commit per Commit object (the light client's Trusting + Light pair)
        for q, (mode, vals, chain_id, block_id, height, commit, num, den) in enumerate(self.requests):
            vs = vcs.get(id(vals))
            if vs is None:
                vs = vcs[id(vals)] = _valset_c(vals, self.keep)
            cc = ccs.get(id(commit))
            if cc is None:
                cc = ccs[id(commit)] = _commit_c(commit, self.keep)
            cid = chain_id.encode()
            bid = _block_id_c(block_id, self.keep) if block_id is not None else None
            self.keep.extend([vs, cc, cid, bid, vals])
            self.reqs[q] = _RequestC(mode, cid, len(cid), ctypes.pointer(vs),
                                     ctypes.pointer(bid) if bid is not None else None, height, ctypes.pointer(cc),
                                     num, den)
        self.res = (_ResultC * max(n, 1))()

    def run(self, engine):
        rc = _bind().tmed_verify_commits(engine._h, self.reqs, self.n, self.res)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_commits")
        return self.res

    def codes(self):
        return np.array([self.res[q].code for q in range(self.n)], np.int32)

    def verified(self):
        return np.array([self.res[q].verified for q in range(self.n)], np.int64)

    def errors(self):
        out = []
        for q, (mode, vals, chain_id, block_id, height, commit, num, den) in enumerate(self.requests):
            out.append(_to_error(self.res[q].code, self.res[q], vals, block_id, commit))
        return out


def seam_phase_us():
    """(plan, verify, replay) wall microseconds of this thread's last seam call (tmed_seam_phase_us)."""
    l = _bind()
    out = (ctypes.c_double * 3)()
    rc = l.tmed_seam_phase_us(out)
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_seam_phase_us")
    return tuple(out)


def run_requests(engine, reqs, n: int, verifier=None):
    """tmed_verify_commits (engine), tmed_verify_commits_multi (a list of engines) or
    tmed_verify_commits_with (verifier: a Python batch verifier, the CPU tests) over n C requests
    already marshalled (a POINTER(_RequestC) or an array of them); returns the _ResultC array."""
    l = _bind()
    res = (_ResultC * max(n, 1))()
    if verifier is None and isinstance(engine, (list, tuple)):  # several GPUs, one process
        rc = l.tmed_verify_commits_multi(_ctx_array(engine), len(engine), reqs, n, res)
    elif verifier is None:
        rc = l.tmed_verify_commits(engine._h, reqs, n, res)
    else:
        def cb(user, pubs, sigs, lens, msgs, offs, m, out):
            try:
                P = ctypes.POINTER(ctypes.c_uint8)
                pa = np.ctypeslib.as_array(ctypes.cast(pubs, P), (m * 32,)).reshape(m, 32)
                sa = np.ctypeslib.as_array(ctypes.cast(sigs, P), (m * 64,)).reshape(m, 64)
                la = np.ctypeslib.as_array(ctypes.cast(lens, ctypes.POINTER(ctypes.c_uint32)), (m,))
                oa = np.ctypeslib.as_array(ctypes.cast(offs, ctypes.POINTER(ctypes.c_uint32)), (m + 1,))
                ma = np.ctypeslib.as_array(ctypes.cast(msgs, P), (int(oa[-1]) + 1,))
                dec = verifier(pa.copy(), sa.copy(), la.copy(), ma.copy(), oa.copy())
                np.ctypeslib.as_array(ctypes.cast(out, P), (m,))[:] = dec
                return 0
            except Exception:  # never raise across the ABI
                return -3
        fn = VERIFY_FN(cb)
        rc = l.tmed_verify_commits_with(reqs, n, res, fn, None)
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_verify_commits")
    return res


def verify_commits(engine, requests: Sequence[tuple], verifier=None, stats: Optional[list] = None):
    """Verify many commits with one device batch.

    requests: (mode, ValidatorSet, chain_id, BlockID|None, height, Commit, trust_num, trust_den).
    engine: an Engine, or a list of Engines (one per GPU: tmed_verify_commits_multi shards the
    requests over them in this process).
    verifier: None -> the engine's GPU path (tmed_verify_commits); otherwise a Python callable
    ``(pubs, sigs, lens, msgs, offs) -> uint8 array`` (used by the CPU test-suite with the oracle).
    Returns one Go-style error (or None) per request.
    """
    l = _bind()
    keep = []
    n = len(requests)
    reqs = (_RequestC * max(n, 1))()
    ccs = {}  # one tmed_commit per Commit object (the light client's Trusting + Light pair)
    vcs = {}  # one tmed_valset per ValidatorSet object: the seam resolves each set once per call
    for q, (mode, vals, chain_id, block_id, height, commit, num, den) in enumerate(requests):
        vs = vcs.get(id(vals))
        if vs is None:
            vs = vcs[id(vals)] = _valset_c(vals, keep)
            keep.append(vals)
        cc = ccs.get(id(commit))
        if cc is None:
            cc = ccs[id(commit)] = _commit_c(commit, keep)
        cid = chain_id.encode()
        bid = _block_id_c(block_id, keep) if block_id is not None else None
        keep.extend([vs, cc, cid, bid])
        reqs[q] = _RequestC(mode, cid, len(cid), ctypes.pointer(vs),
                            ctypes.pointer(bid) if bid is not None else None, height, ctypes.pointer(cc), num, den)
    res = run_requests(engine, reqs, n, verifier)
    out = []
    for q, (mode, vals, chain_id, block_id, height, commit, num, den) in enumerate(requests):
        out.append(_to_error(res[q].code, res[q], vals, block_id, commit))
        if stats is not None:
            stats.append(int(res[q].verified))
    return out


class BlocksyncWindow:
    """A window of blocks for the blocksync reactor (f4; blockchain/v0/reactor.go:349-418):
    block h is checked with vals.VerifyCommitLight(chain_id, block_ids[h], heights[h], commits[h]).
    Packed into C structs once; run() verifies the whole window speculatively through the
    pipelined device path (tmed_blocksync_verify) and returns the C results."""

    def __init__(self, vals: "ValidatorSet", chain_id: str, block_ids: Sequence[BlockID], heights: Sequence[int],
                 commits: Sequence):
        n = len(commits)
        self.n, self.vals, self.block_ids, self.commits = n, vals, list(block_ids), list(commits)
        self.keep = []
        self.vs = _valset_c(vals, self.keep)
        self.bids = (_BlockIDC * max(n, 1))()
        self.ccs = (_CommitC * max(n, 1))()
        for h in range(n):
            self.bids[h] = _block_id_c(self.block_ids[h], self.keep)
            self.ccs[h] = _commit_c(self.commits[h], self.keep)
        self.heights = np.ascontiguousarray(np.asarray(heights, np.int64).reshape(max(n, 0)))
        self.cid = chain_id.encode()
        self.win = _BlocksyncWindowC(self.cid, len(self.cid), ctypes.pointer(self.vs), n, self.bids,
                                     _ptr(self.heights), self.ccs)
        self.res = (_ResultC * max(n, 1))()

    def run(self, engine, batch_blocks: int = 0):
        """engine: one Engine, or a list of Engines (one per GPU): the window is sharded over them."""
        if isinstance(engine, (list, tuple)):
            rc = _bind().tmed_blocksync_verify_multi(_ctx_array(engine), len(engine), ctypes.byref(self.win),
                                                     batch_blocks, self.res)
        else:
            rc = _bind().tmed_blocksync_verify(engine._h, ctypes.byref(self.win), batch_blocks, self.res)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_blocksync_verify")
        return self.res

    def submit(self, engine, batch_blocks: int = 0):
        """tmed_blocksync_submit: queue this window behind the engine's windows in flight; returns
        once every EARLIER submitted window's results are final (this one's are final after the
        next submit or blocksync_wait).  The window's commit arrays must stay unchanged until then."""
        rc = _bind().tmed_blocksync_submit(engine._h, ctypes.byref(self.win), batch_blocks, self.res)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_blocksync_submit")
        return self.res

    def codes(self):
        return np.array([self.res[h].code for h in range(self.n)], np.int32)

    def verified(self):
        return np.array([self.res[h].verified for h in range(self.n)], np.int64)

    def errors(self):
        return [_to_error(self.res[h].code, self.res[h], self.vals, self.block_ids[h], self.commits[h])
                for h in range(self.n)]
