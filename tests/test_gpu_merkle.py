"""GPU parity for the batched Merkle kernels (f3) vs oracle/merkle.py (bit-exact roots)."""
import hashlib
import random

import numpy as np
import pytest

from oracle import merkle as M
from test_merkle_oracle import KAT_HEADER_HASH, TREE_KATS, kat_header

pytestmark = pytest.mark.gpu


def test_tree_kats_gpu(engine):
    from tmed.merkle import merkle_roots
    got = merkle_roots(engine, [items for items, _ in TREE_KATS])
    assert [g.hex() for g in got] == [e for _, e in TREE_KATS]


def test_random_forest_gpu(engine):
    """Many trees of 0..300 leaves, leaf lengths 0..200 (every misalignment of the word
    reader), in one call: exactly the oracle's roots."""
    from tmed.merkle import merkle_roots
    rng = random.Random(21)
    trees = []
    for n in list(range(0, 70)) + [127, 128, 129, 255, 256, 257, 300]:
        trees.append([rng.randbytes(rng.randrange(0, 200)) for _ in range(n)])
    got = merkle_roots(engine, trees)
    for t, g in zip(trees, got):
        assert g == M.hash_from_byte_slices(t), len(t)


def test_valset_hashes_gpu(engine):
    """ValidatorSet.Hash over SimpleValidator leaves: powers 0, small, 2^62, negative (10-byte
    varint), set sizes 0..400 — vs the oracle; plus the empty-set vector of the reference."""
    from tmed.merkle import valset_hashes_arrays
    rng = np.random.default_rng(5)
    sizes = [0, 1, 2, 3, 7, 64, 175, 400]
    n = sum(sizes)
    pubs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    powers = rng.integers(0, 1 << 40, n, dtype=np.int64)
    powers[::7] = 0
    powers[1::11] = (1 << 62) - 1
    powers[2::13] = -5
    off = np.zeros(len(sizes) + 1, np.uint32)
    off[1:] = np.cumsum(sizes)
    got = valset_hashes_arrays(engine, pubs, powers, off)
    for s in range(len(sizes)):
        vals = [(bytes(pubs[i]), int(powers[i])) for i in range(off[s], off[s + 1])]
        assert bytes(got[s]) == M.valset_hash(vals), sizes[s]
    assert bytes(got[0]).hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"


def test_header_hashes_gpu(engine):
    from tmed.merkle import header_hashes
    rng = random.Random(3)
    hs = [kat_header()]
    for i in range(300):
        h = kat_header()
        h["height"] = rng.choice([0, 1, 3, 2**40, 2**63 - 1])
        h["chain_id"] = rng.choice(["", "c", "test_chain_id", "x" * 50])
        h["time"] = (rng.choice([0, -62135596800, 1700000000 + i]), rng.choice([0, 1, 999999999]))
        h["version_block"], h["version_app"] = rng.choice([0, 11]), rng.choice([0, 1, 2**33])
        h["last_block_id"] = (rng.choice([b"", rng.randbytes(32)]), rng.choice([0, 1, 6, 300]),
                              rng.choice([b"", rng.randbytes(32)]))
        for k in M.HEADER_HASH_FIELDS:
            if rng.random() < 0.2:
                h[k] = b""
        hs.append(h)
    got = header_hashes(engine, hs)
    assert got[0].hex().upper() == KAT_HEADER_HASH
    for h, g in zip(hs, got):
        assert g == M.header_hash(h)
    assert any(g is None for g in got)


@pytest.mark.parametrize("part_size", [64, 100, 65536])
def test_partset_roots_gpu(engine, part_size):
    from tmed.merkle import partset_roots
    rng = random.Random(part_size)
    blocks = [b"", b"\x01", rng.randbytes(part_size - 1), rng.randbytes(part_size), rng.randbytes(part_size + 1),
              rng.randbytes(7 * part_size // 2), rng.randbytes(3 * 65536 + 17)]
    got = partset_roots(engine, blocks, part_size)
    for b, g in zip(blocks, got):
        assert g == M.partset_root(b, part_size), len(b)
