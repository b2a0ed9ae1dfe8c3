"""Batched Merkle hashing on the GPU — host mirror of the reference's
``crypto/merkle.HashFromByteSlices`` (crypto/merkle/tree.go:9-22), ``ValidatorSet.Hash``
(types/validator_set.go:347-353), ``Header.Hash`` (types/block.go:440-475) and the
``PartSet`` root (types/part_set.go:166-194), each over many objects per call through the
C ABI (csrc/merkle.hip).  Same inputs and outputs as the Go functions, one list entry per
object; ``Header.Hash``'s nil is ``None``."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from ._native import TMED_OK, TmedError, lib

BLOCK_PART_SIZE_BYTES = 65536  # types/params.go:19 BlockPartSizeBytes


class _HeaderBlockID(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_void_p), ("hash_len", ctypes.c_uint32), ("psh_total", ctypes.c_uint32),
                ("psh_hash", ctypes.c_void_p), ("psh_hash_len", ctypes.c_uint32)]


class _HeaderC(ctypes.Structure):
    _fields_ = [("version_block", ctypes.c_uint64), ("version_app", ctypes.c_uint64),
                ("chain_id", ctypes.c_char_p), ("chain_id_len", ctypes.c_uint32), ("height", ctypes.c_int64),
                ("time_seconds", ctypes.c_int64), ("time_nanos", ctypes.c_int32), ("last_block_id", _HeaderBlockID),
                ("hashes", ctypes.c_void_p * 9), ("hash_lens", ctypes.c_uint32 * 9)]


HEADER_HASH_FIELDS = ("last_commit_hash", "data_hash", "validators_hash", "next_validators_hash",
                      "consensus_hash", "app_hash", "last_results_hash", "evidence_hash", "proposer_address")


def _bind():
    l = lib()
    if l.tmed_merkle_roots.argtypes is None:
        P, SZ = ctypes.c_void_p, ctypes.c_size_t
        l.tmed_merkle_roots.restype = ctypes.c_int
        l.tmed_merkle_roots.argtypes = [P, P, P, P, SZ, P]
        l.tmed_valset_hashes.restype = ctypes.c_int
        l.tmed_valset_hashes.argtypes = [P, P, P, P, SZ, P]
        l.tmed_header_hashes.restype = ctypes.c_int
        l.tmed_header_hashes.argtypes = [P, ctypes.POINTER(_HeaderC), SZ, P, P]
        l.tmed_partset_roots.restype = ctypes.c_int
        l.tmed_partset_roots.argtypes = [P, P, P, SZ, ctypes.c_uint32, P]
    return l


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def merkle_roots(engine, trees: Sequence[Sequence[bytes]]) -> list:
    """HashFromByteSlices(tree) for every tree (list of byte-slice lists)."""
    flat, leaf_lens, counts = [], [], []
    for t in trees:
        counts.append(len(t))
        for leaf in t:
            flat.append(bytes(leaf))
            leaf_lens.append(len(leaf))
    leaf_off = np.zeros(len(leaf_lens) + 1, np.uint64)
    np.cumsum(np.asarray(leaf_lens, np.uint64), out=leaf_off[1:])
    tree_off = np.zeros(len(counts) + 1, np.uint32)
    np.cumsum(np.asarray(counts, np.uint32), out=tree_off[1:])
    data = np.frombuffer(b"".join(flat) + b"\0" * 8, np.uint8)
    roots = np.zeros((max(len(trees), 1), 32), np.uint8)
    if not trees:
        return []
    rc = _bind().tmed_merkle_roots(engine._h, _p(data), _p(leaf_off), _p(tree_off), len(trees), _p(roots))
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_merkle_roots")
    return [bytes(r) for r in roots[:len(trees)]]


def valset_hashes_arrays(engine, pubkeys: np.ndarray, powers: np.ndarray, set_off: np.ndarray) -> np.ndarray:
    """ValidatorSet.Hash of sets [set_off[s], set_off[s+1]) over (pubkeys u8[N,32], powers i64[N])."""
    n_sets = set_off.shape[0] - 1
    out = np.zeros((max(n_sets, 1), 32), np.uint8)
    if n_sets <= 0:
        return out[:0]
    pk = np.ascontiguousarray(pubkeys, np.uint8).reshape(-1, 32)
    pw = np.ascontiguousarray(powers, np.int64)
    so = np.ascontiguousarray(set_off, np.uint32)
    rc = _bind().tmed_valset_hashes(engine._h, _p(pk) if pk.size else None, _p(pw) if pw.size else None, _p(so),
                                    n_sets, _p(out))
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_valset_hashes")
    return out[:n_sets]


def valset_hashes(engine, valsets: Sequence) -> list:
    """ValidatorSet.Hash() of every tmed.types.ValidatorSet (ed25519 validators)."""
    pubs, pows, off = [], [], [0]
    for vs in valsets:
        for v in vs.validators:
            pubs.append(np.frombuffer(v.pub_key, np.uint8))
            pows.append(v.voting_power)
        off.append(len(pubs))
    pk = np.array(pubs, np.uint8).reshape(-1, 32) if pubs else np.zeros((0, 32), np.uint8)
    return [bytes(r) for r in valset_hashes_arrays(engine, pk, np.array(pows, np.int64), np.array(off, np.uint32))]


class HeaderBatch:
    """Headers packed into C structs once (repeated timing of the C call alone)."""

    def __init__(self, headers: Sequence[dict]):
        n = self.n = len(headers)
        self.hs = (_HeaderC * max(n, 1))()
        self.keep = []
        for i, h in enumerate(headers):
            cid = h["chain_id"].encode()
            bh, pt, ph = h["last_block_id"]
            bh, ph = bytes(bh), bytes(ph)
            self.keep.extend([cid, bh, ph])
            c = self.hs[i]
            c.version_block, c.version_app = h["version_block"], h["version_app"]
            c.chain_id, c.chain_id_len = cid, len(cid)
            c.height = h["height"]
            c.time_seconds, c.time_nanos = h["time"]
            c.last_block_id = _HeaderBlockID(ctypes.cast(ctypes.c_char_p(bh), ctypes.c_void_p), len(bh), pt,
                                             ctypes.cast(ctypes.c_char_p(ph), ctypes.c_void_p), len(ph))
            for k, name in enumerate(HEADER_HASH_FIELDS):
                v = bytes(h[name])
                self.keep.append(v)
                c.hashes[k] = ctypes.cast(ctypes.c_char_p(v), ctypes.c_void_p)
                c.hash_lens[k] = len(v)
        self.out = np.zeros((max(n, 1), 32), np.uint8)
        self.ok = np.zeros(max(n, 1), np.uint8)

    def run(self, engine) -> list:
        if self.n == 0:
            return []
        rc = _bind().tmed_header_hashes(engine._h, self.hs, self.n, _p(self.out), _p(self.ok))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_header_hashes")
        return [bytes(self.out[i]) if self.ok[i] else None for i in range(self.n)]


def header_hashes(engine, headers: Sequence[dict]) -> list:
    """Header.Hash of every header (dict with the fields of oracle/merkle.py's header_leaves);
    None where the reference returns nil (empty ValidatorsHash)."""
    return HeaderBatch(headers).run(engine)


def partset_roots_packed(engine, data: np.ndarray, off: np.ndarray, part_size: int = BLOCK_PART_SIZE_BYTES):
    """Roots of blocks data[off[b] .. off[b+1]) (u8 array, u64 offsets): an n x 32 array."""
    n = off.shape[0] - 1
    roots = np.zeros((max(n, 1), 32), np.uint8)
    if n <= 0:
        return roots[:0]
    rc = _bind().tmed_partset_roots(engine._h, _p(data), _p(np.ascontiguousarray(off, np.uint64)), n, part_size,
                                    _p(roots))
    if rc != TMED_OK:
        raise TmedError(rc, "tmed_partset_roots")
    return roots[:n]


def partset_roots(engine, blocks: Sequence[bytes], part_size: int = BLOCK_PART_SIZE_BYTES) -> list:
    """NewPartSetFromData(block, part_size).Hash() for every block's bytes."""
    n = len(blocks)
    if n == 0:
        return []
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(np.asarray([len(b) for b in blocks], np.uint64), out=off[1:])
    data = np.frombuffer(b"".join(bytes(b) for b in blocks) + b"\0" * 8, np.uint8)
    return [bytes(r) for r in partset_roots_packed(engine, data, off, part_size)]
