"""CanonicalVote sign-bytes through the library (tmed_vote_sign_bytes).

Product-side counterpart of ``Commit.VoteSignBytes`` (reference
``types/block.go:807-810`` -> ``types/vote.go:93-101``); see
``csrc/signbytes.hip`` for the byte layout and citations.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import TMED_OK, TmedError, lib

ZERO_TIME = (-62135596800, 0)  # Go's zero time.Time (types/vote_test.go:70)


class VoteTemplate(ctypes.Structure):
    _fields_ = [("chain_id", ctypes.c_char_p), ("chain_id_len", ctypes.c_uint32),
                ("height", ctypes.c_int64), ("round", ctypes.c_int32),
                ("block_hash", ctypes.c_char_p), ("block_hash_len", ctypes.c_uint32),
                ("psh_total", ctypes.c_uint32),
                ("psh_hash", ctypes.c_char_p), ("psh_hash_len", ctypes.c_uint32)]


def _bind():
    l = lib()
    f = l.tmed_vote_sign_bytes
    if f.argtypes is None:
        P = ctypes.c_void_p
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.POINTER(VoteTemplate), ctypes.c_size_t, P, P, P, P, ctypes.c_size_t, P,
                      ctypes.POINTER(ctypes.c_size_t)]
    return f


def make_template(chain_id: str, height: int, round_: int, block_hash: bytes = b"", psh_total: int = 0,
                  psh_hash: bytes = b"") -> VoteTemplate:
    cid = chain_id.encode()
    t = VoteTemplate(cid, len(cid), height, round_, block_hash, len(block_hash), psh_total, psh_hash, len(psh_hash))
    t._keep = (cid, block_hash, psh_hash)  # keep the buffers alive
    return t


def vote_sign_bytes_batch(t: VoteTemplate, ts_seconds, ts_nanos, flags=None):
    """Sign-bytes of n votes of one commit -> (flat u8 array, u32 offsets[n+1])."""
    f = _bind()
    sec = np.ascontiguousarray(ts_seconds, dtype=np.int64)
    nan = np.ascontiguousarray(ts_nanos, dtype=np.int32)
    n = sec.shape[0]
    fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
    off = np.zeros(n + 1, np.uint32)
    total = ctypes.c_size_t(0)
    P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = f(ctypes.byref(t), n, P(fl), P(sec), P(nan), None, 0, P(off), ctypes.byref(total))
    if rc not in (TMED_OK,):
        raise TmedError(rc, "tmed_vote_sign_bytes(size)")
    out = np.zeros(max(1, total.value), np.uint8)
    rc = f(ctypes.byref(t), n, P(fl), P(sec), P(nan), P(out), out.shape[0], P(off), ctypes.byref(total))
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_vote_sign_bytes")
    return out[:total.value], off


def vote_sign_bytes(chain_id: str, height: int, round_: int, block_id, timestamp, flag: int = 2) -> bytes:
    """One vote (convenience for tests): block_id = (hash, psh_total, psh_hash)."""
    bh, pt, ph = block_id if block_id is not None else (b"", 0, b"")
    t = make_template(chain_id, height, round_, bh, pt, ph)
    flat, off = vote_sign_bytes_batch(t, [timestamp[0]], [timestamp[1]], [flag])
    return flat[off[0]:off[1]].tobytes()
