"""Synthetic workloads of BASELINE.json, built with the product's own signer.

C2: n signatures, each with its own key
  seed_i  = SHA-512("tmed-c2" || LE64(i))[:32]
  M_i     = CanonicalVote sign-bytes: height = 1 + i // 175, round 0,
            chain "test_chain_id", BlockID hash = SHA-256(LE64(height)),
            PSH {total 123, hash = SHA-256("psh" || LE64(height))},
            timestamp 2023-01-01T00:00:00Z + (i % 175) ms
Signatures and public keys are produced on the GPU by the RFC 8032 signer
kernel (the same code the parity tests check against the oracle).
"""
from __future__ import annotations

import hashlib

import numpy as np

from .signbytes import make_template, vote_sign_bytes_batch

T2023 = 1672531200  # 2023-01-01T00:00:00Z
VALS_PER_COMMIT = 175


def c2_seeds(start: int, n: int) -> np.ndarray:
    out = np.empty((n, 32), np.uint8)
    for j in range(n):
        out[j] = np.frombuffer(hashlib.sha512(b"tmed-c2" + (start + j).to_bytes(8, "little")).digest()[:32], np.uint8)
    return out


def c2_messages(start: int, n: int, chain_id: str = "test_chain_id"):
    """Sign-bytes for signatures start..start+n-1 -> (flat u8, u32 offsets)."""
    parts, offs = [], [np.zeros(1, np.uint32)]
    base = 0
    i = start
    end = start + n
    while i < end:
        h = 1 + i // VALS_PER_COMMIT
        j_end = min(end, (h) * VALS_PER_COMMIT)
        k = np.arange(i, j_end)
        t = make_template(chain_id, h, 0, hashlib.sha256(h.to_bytes(8, "little")).digest(), 123,
                          hashlib.sha256(b"psh" + h.to_bytes(8, "little")).digest())
        flat, off = vote_sign_bytes_batch(t, np.full(k.shape[0], T2023, np.int64),
                                          ((k % VALS_PER_COMMIT) * 1_000_000).astype(np.int32))
        parts.append(flat)
        offs.append(off[1:] + base)
        base += int(off[-1])
        i = j_end
    return np.concatenate(parts), np.concatenate(offs).astype(np.uint32)
