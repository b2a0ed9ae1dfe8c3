"""ctypes face of shim/go_marshal.cpp (libtmed_gomarshal.so): the cgo shim's host marshal in compiled
code, over commits and validator sets laid out as Go 1.18 holds them (types/block.go:595-600,
737-752; types/validator_set.go:51-58).  The benches build those objects once (GoHeap, untimed)
and time Marshal.window / Marshal.requests beside the seam: what a drop-in caller pays on the host
before tmed_blocksync_submit / tmed_verify_commits.  Host-only (no GPU call)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import types as T

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG, "lib", "libtmed_gomarshal.so")
_lib = None


def _l():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("%s is missing: make -C tendermint-fork_amd" % LIB_PATH)
        l = ctypes.CDLL(LIB_PATH)
        P, SZ, I64, I32, U32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32
        l.gm_heap_new.restype = P
        l.gm_heap_new.argtypes = []
        l.gm_heap_free.restype = None
        l.gm_heap_free.argtypes = [P]
        l.go_commit_build.restype = I64
        l.go_commit_build.argtypes = [P, I64, I32, P, U32, U32, P, U32, SZ, P, P, P, P, P, P, P]
        l.go_valset_build.restype = I64
        l.go_valset_build.argtypes = [P, SZ, P, P, P]
        l.gm_ctx_new.restype = P
        l.gm_ctx_new.argtypes = [ctypes.c_int]
        l.gm_ctx_free.restype = None
        l.gm_ctx_free.argtypes = [P]
        l.gm_forget_sets.restype = None
        l.gm_forget_sets.argtypes = [P]
        l.gm_marshal_window.restype = ctypes.POINTER(T._BlocksyncWindowC)
        l.gm_marshal_window.argtypes = [P, P, I64, P, P, SZ, ctypes.c_char_p, U32, P, P]
        l.gm_marshal_requests.restype = ctypes.POINTER(T._RequestC)
        l.gm_marshal_requests.argtypes = [P, P, SZ, P, P, P, P, P, P, ctypes.c_char_p, U32, P]
        _lib = l
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class GoHeap:
    """Commits and validator sets as Go objects (slice headers, per-signature heap objects,
    interface-held public keys); indices returned by commit() / valset()."""

    def __init__(self):
        self.h = _l().gm_heap_new()

    def commit(self, pc: "T.PackedCommit") -> int:
        b = pc.block_id
        keep = [np.ascontiguousarray(x) for x in (pc.flags, pc.addresses, pc.ts_seconds, pc.ts_nanos, pc.sigs,
                                                  pc.sig_lens)]
        keep = [keep[0].astype(np.uint8, copy=False), keep[1].astype(np.uint8, copy=False),
                keep[2].astype(np.int64, copy=False), keep[3].astype(np.int32, copy=False),
                keep[4].astype(np.uint8, copy=False), keep[5].astype(np.uint32, copy=False)]
        al = None if pc.address_lens is None else np.ascontiguousarray(pc.address_lens, np.uint32)
        h = np.frombuffer(bytes(b.hash) + b"\0", np.uint8)
        ph = np.frombuffer(bytes(b.psh_hash) + b"\0", np.uint8)
        return _l().go_commit_build(self.h, pc.height, pc.round, _p(h), h.size - 1, b.psh_total, _p(ph), ph.size - 1,
                                    keep[0].shape[0],
                                    _p(keep[0]), _p(keep[1]), _p(al), _p(keep[2]), _p(keep[3]), _p(keep[4]),
                                    _p(keep[5]))

    def valset(self, vals: "T.ValidatorSet") -> int:
        pubs, powers, addrs = vals.packed()
        return _l().go_valset_build(self.h, len(vals.validators), _p(pubs), _p(powers), _p(addrs))

    def free(self):
        if self.h:
            _l().gm_heap_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Marshal:
    """One shim marshal context: reusable C buffers (a window in flight needs its own context: the
    library reads the window's arrays until its results are final)."""

    def __init__(self, threads: int | None = None):
        t = threads or int(os.environ.get("TMED_HOST_THREADS", "16"))
        self.c = _l().gm_ctx_new(t)

    def window(self, heap: GoHeap, set_idx: int, commit_idx, heights, chain_id: str, set_hash=None, sig_arena=None):
        """-> POINTER(_BlocksyncWindowC) for tmed_blocksync_submit / _verify (valid until the next call)."""
        ci = np.ascontiguousarray(commit_idx, np.int64)
        hs = np.ascontiguousarray(heights, np.int64)
        cid = chain_id.encode()
        sh = None if set_hash is None else np.frombuffer(bytes(set_hash), np.uint8)
        self._keep = (ci, hs, cid, sh)
        return _l().gm_marshal_window(self.c, heap.h, set_idx, _p(ci), _p(hs), ci.shape[0], cid, len(cid), _p(sh),
                                      sig_arena)

    def requests(self, heap: GoHeap, modes, set_idx, commit_idx, heights, tnum, tden, chain_id: str,
                 set_hashes=None, forget_sets: bool = True):
        """-> POINTER(_RequestC) of len(modes) requests.  forget_sets: flatten every set again (a new
        light-client batch: the shim's per-*ValSet cache starts empty)."""
        if forget_sets:
            _l().gm_forget_sets(self.c)
        arrs = (np.ascontiguousarray(modes, np.int32), np.ascontiguousarray(set_idx, np.int64),
                np.ascontiguousarray(commit_idx, np.int64), np.ascontiguousarray(heights, np.int64),
                np.ascontiguousarray(tnum, np.int64), np.ascontiguousarray(tden, np.int64))
        cid = chain_id.encode()
        sh = None if set_hashes is None else np.ascontiguousarray(set_hashes, np.uint8)
        self._keep = (arrs, cid, sh)
        return _l().gm_marshal_requests(self.c, heap.h, arrs[0].shape[0], *[_p(a) for a in arrs], cid, len(cid),
                                        _p(sh))

    def free(self):
        if self.c:
            _l().gm_ctx_free(self.c)
            self.c = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def results(n: int):
    return (T._ResultC * max(n, 1))()


def packed_of(c) -> "T.PackedCommit":
    """A T.Commit (CommitSig objects) as the arrays GoHeap.commit takes (PackedCommits pass through)."""
    if isinstance(c, T.PackedCommit):
        return c
    n = len(c.signatures)
    flags = np.zeros(n, np.uint8)
    addrs = np.zeros((n, 20), np.uint8)
    alens = np.zeros(n, np.uint32)
    sec = np.zeros(n, np.int64)
    nsec = np.zeros(n, np.int32)
    sigs = np.zeros((n, 64), np.uint8)
    slens = np.zeros(n, np.uint32)
    for i, cs in enumerate(c.signatures):
        flags[i] = cs.flag
        a = bytes(cs.address)[:20]
        addrs[i, :len(a)] = np.frombuffer(a, np.uint8)
        alens[i] = len(cs.address)
        sec[i], nsec[i] = cs.timestamp
        s = bytes(cs.signature)[:64]
        sigs[i, :len(s)] = np.frombuffer(s, np.uint8)
        slens[i] = len(cs.signature)
    return T.PackedCommit(c.height, c.round, c.block_id, flags, addrs, sec, nsec, sigs, slens, alens)
