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


# ----------------------------------------------------------------------------- commits (C1, C3, C4)

def seeds_from_tag(tag: bytes, start: int, n: int) -> np.ndarray:
    out = np.empty((n, 32), np.uint8)
    for j in range(n):
        out[j] = np.frombuffer(hashlib.sha256(tag + (start + j).to_bytes(8, "little")).digest(), np.uint8)
    return out


def pubkeys_of(engine, seeds: np.ndarray) -> np.ndarray:
    """ed25519 public keys of seeds (GPU RFC 8032 key derivation)."""
    n = seeds.shape[0]
    _, pubs = engine.sign_arrays(seeds, np.zeros(16, np.uint8), np.zeros(n + 1, np.uint32))
    return pubs


def make_valset(pubs: np.ndarray, powers):
    """ValidatorSet sorted like types.ValidatorsByVotingPower (power desc, address asc,
    types/validator_set.go:906-911); returns (vals, order) with order[i] = input index of validator i."""
    from .types import Validator, ValidatorSet, address_of
    items = [(int(powers[i]), address_of(pubs[i].tobytes()), i) for i in range(pubs.shape[0])]
    items.sort(key=lambda t: (-t[0], t[1]))
    vals = ValidatorSet([Validator(pubs[i].tobytes(), p, 0, a) for p, a, i in items])
    return vals, np.array([i for _, _, i in items], np.int64)


def sign_commits(engine, chain_id: str, specs, sign_upto: int | None = None):
    """specs: list of (seeds_in_validator_order u8[n,32], addresses u8[n,20], height, round, BlockID,
    ts_base_seconds, flags or None).  All votes of all commits are signed in ONE GPU call.
    Returns a list of PackedCommit (timestamps: base + i ms for validator i).
    sign_upto: only validators [0, sign_upto) sign; the others' signatures are filled with
    seeded random bytes (present, flag Commit, invalid) — for workloads whose loop provably
    stops before them (VerifyCommitLight at equal powers stops after 2n/3+1 signatures)."""
    from .types import PackedCommit
    flats, offs, seeds_all, metas = [], [], [], []
    base = 0
    for seeds, addrs, height, round_, bid, ts0, flags in specs:
        n = seeds.shape[0]
        t = make_template(chain_id, height, round_, bid.hash, bid.psh_total, bid.psh_hash)
        sec = np.full(n, ts0, np.int64) + (np.arange(n) // 1000)
        nan = ((np.arange(n) % 1000) * 1_000_000).astype(np.int32)
        fl = np.full(n, 2, np.uint8) if flags is None else np.asarray(flags, np.uint8)
        ns = n if sign_upto is None else min(n, sign_upto)
        f, o = vote_sign_bytes_batch(t, sec[:ns], nan[:ns], fl[:ns])
        flats.append(f)
        offs.append(o[:-1].astype(np.int64) + base)
        base += int(o[-1])
        seeds_all.append(seeds[:ns])
        metas.append((height, round_, bid, addrs, sec, nan, fl, ns))
    flat = np.concatenate(flats) if flats else np.zeros(0, np.uint8)
    off = np.concatenate(offs + [np.array([base], np.int64)]).astype(np.uint32)
    sigs, _ = engine.sign_arrays(np.concatenate(seeds_all), np.concatenate([flat, np.zeros(16, np.uint8)]), off)
    out, k = [], 0
    rng = np.random.default_rng(0x5EED)
    for (height, round_, bid, addrs, sec, nan, fl, ns) in metas:
        n = sec.shape[0]
        s = np.empty((n, 64), np.uint8)
        s[:ns] = sigs[k:k + ns]
        if ns < n:
            s[ns:] = rng.integers(0, 256, (n - ns, 64), dtype=np.uint8)
        lens = np.full(n, 64, np.uint32)
        absent = fl == 1
        s[absent] = 0
        lens[absent] = 0
        a = addrs.copy()
        a[absent] = 0
        out.append(PackedCommit(height, round_, bid, fl, a, sec, nan, s, lens))
        k += ns
    return out


# The eight small-order points of edwards25519 (canonical encodings, and the two with the
# x = 0 sign bit set): public constants, the same set as the oracle's small_order_points().
SMALL_ORDER = [bytes.fromhex(h) for h in (
    "0100000000000000000000000000000000000000000000000000000000000000",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa")]
_L = 2 ** 252 + 27742317777372353535851937790883648493
_P = 2 ** 255 - 19


def c5_mix(pubs: np.ndarray, sigs: np.ndarray, seed: int = 0x5EED, frac: float = 0.01) -> np.ndarray:
    """BASELINE C5 in place: `frac` of the tuples (uniform, seeded) replaced, cycling over the
    edge classes of SURVEY §8c — R/S/M bit flip, S + L, small-order A, small-order R,
    non-canonical A (y = p + small), R sign flip.  Returns the modified indices."""
    n = pubs.shape[0]
    rng = np.random.default_rng(seed)
    idx = rng.choice(n, int(n * frac), replace=False)
    for j, i in enumerate(idx):
        k = j % 6
        if k == 0:
            sigs[i, rng.integers(0, 64)] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif k == 1:
            s = int.from_bytes(sigs[i, 32:].tobytes(), "little") + _L
            sigs[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif k == 2:
            pubs[i] = np.frombuffer(SMALL_ORDER[j % 8], np.uint8)
        elif k == 3:
            sigs[i, :32] = np.frombuffer(SMALL_ORDER[j % 8], np.uint8)
        elif k == 4:
            pubs[i] = np.frombuffer((int(rng.integers(0, 19)) + _P).to_bytes(32, "little"), np.uint8)
        else:
            sigs[i, 31] ^= np.uint8(0x80)
    return idx
