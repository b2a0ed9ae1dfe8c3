"""RFC-6962 Merkle hashing restatement (TEST INFRASTRUCTURE ONLY).

Follows, line for line:
* ``crypto/merkle/tree.go:9-22``      HashFromByteSlices (recursive, split at the largest power
  of two strictly below n, ``getSplitPoint``)
* ``crypto/merkle/hash.go:13-27``     emptyHash / leafHash (0x00 prefix) / innerHash (0x01 prefix),
  tmhash = SHA-256 (``crypto/tmhash/hash.go:19-22``)
* ``types/validator_set.go:347-353``  ValidatorSet.Hash over Validator.Bytes()
* ``types/validator.go:117-133``      Validator.Bytes = SimpleValidator{PubKey, VotingPower} proto
  (``proto/tendermint/types/validator.pb.go``: pub_key = 1 message, voting_power = 2 int64;
  ``proto/tendermint/crypto/keys.pb.go``: PublicKey oneof ed25519 = 1 bytes)
* ``types/block.go:440-475``          Header.Hash over 14 encoded fields (cdcEncode wrappers,
  ``types/encoding_helper.go``; Version ``proto/tendermint/version/types.pb.go:238-254``;
  BlockID ``proto/tendermint/types/types.pb.go:1153-1256``; gogoproto StdTime)
* ``types/part_set.go:166-194``       NewPartSetFromData root (ProofsFromByteSlices, proof.go:35-48,
  same recursion as HashFromByteSlices)

Pinned by the reference's own known answers: ``crypto/merkle/tree_test.go:22-44`` (six
HashFromByteSlices vectors), ``types/block_test.go:305-326`` (Header.Hash), and
``types/validator_set_test.go:49-51`` (empty set hash).
"""
from __future__ import annotations

import hashlib

from .signbytes import uvarint


def tmhash(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def empty_hash() -> bytes:
    return tmhash(b"")


def leaf_hash(leaf: bytes) -> bytes:
    return tmhash(b"\x00" + leaf)


def inner_hash(left: bytes, right: bytes) -> bytes:
    return tmhash(b"\x01" + left + right)


def split_point(n: int) -> int:
    """getSplitPoint (crypto/merkle/tree.go): largest power of two strictly less than n."""
    if n < 1:
        raise ValueError("Trying to split a tree with size < 1")
    k = 1 << (n.bit_length() - 1)
    return k >> 1 if k == n else k


def hash_from_byte_slices(items) -> bytes:
    n = len(items)
    if n == 0:
        return empty_hash()
    if n == 1:
        return leaf_hash(bytes(items[0]))
    k = split_point(n)
    return inner_hash(hash_from_byte_slices(items[:k]), hash_from_byte_slices(items[k:]))


def hash_from_byte_slices_iterative(items) -> bytes:
    """HashFromByteSlicesIterative (tree.go:57-101): level-by-level pairing, odd node promoted."""
    level = [leaf_hash(bytes(x)) for x in items]
    if not level:
        return empty_hash()
    while len(level) > 1:
        nxt = [inner_hash(level[i], level[i + 1]) for i in range(0, len(level) - 1, 2)]
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    return level[0]


def _bytes_field(tag: int, payload: bytes) -> bytes:
    return bytes([tag]) + uvarint(len(payload)) + payload


def simple_validator_bytes(pub: bytes, power: int) -> bytes:
    """Validator.Bytes() for an ed25519 key."""
    pk = _bytes_field(0x0A, pub)                     # PublicKey{ed25519: pub}
    out = _bytes_field(0x0A, pk)                     # SimpleValidator.pub_key
    if power != 0:
        out += b"\x10" + uvarint(power)              # SimpleValidator.voting_power
    return out


def valset_hash(validators) -> bytes:
    """validators: [(pub32, power)] in set order."""
    return hash_from_byte_slices([simple_validator_bytes(p, w) for p, w in validators])


def header_leaves(h: dict) -> list:
    """The 14 byte slices of Header.Hash.  h keys: version_block, version_app, chain_id, height,
    time (seconds, nanos), last_block_id (hash, psh_total, psh_hash), last_commit_hash, data_hash,
    validators_hash, next_validators_hash, consensus_hash, app_hash, last_results_hash,
    evidence_hash, proposer_address."""
    ver = b""
    if h["version_block"]:
        ver += b"\x08" + uvarint(h["version_block"])
    if h["version_app"]:
        ver += b"\x10" + uvarint(h["version_app"])
    cid = h["chain_id"].encode()
    leaves = [ver, _bytes_field(0x0A, cid) if cid else b""]
    leaves.append(b"\x08" + uvarint(h["height"]) if h["height"] else b"")
    sec, nanos = h["time"]
    ts = b""
    if sec:
        ts += b"\x08" + uvarint(sec)
    if nanos:
        ts += b"\x10" + uvarint(nanos)
    leaves.append(ts)
    bh, pt, ph = h["last_block_id"]
    psh = b""
    if pt:
        psh += b"\x08" + uvarint(pt)
    if ph:
        psh += _bytes_field(0x12, ph)
    bid = (_bytes_field(0x0A, bh) if bh else b"") + _bytes_field(0x12, psh)
    leaves.append(bid)
    for k in HEADER_HASH_FIELDS:
        v = h[k]
        leaves.append(_bytes_field(0x0A, v) if v else b"")
    return leaves


HEADER_HASH_FIELDS = ("last_commit_hash", "data_hash", "validators_hash", "next_validators_hash",
                      "consensus_hash", "app_hash", "last_results_hash", "evidence_hash", "proposer_address")


def header_hash(h: dict):
    """Header.Hash: None (Go nil) when ValidatorsHash is empty."""
    if not h["validators_hash"]:
        return None
    return hash_from_byte_slices(header_leaves(h))


def partset_root(data: bytes, part_size: int) -> bytes:
    parts = [data[i:i + part_size] for i in range(0, len(data), part_size)]
    return hash_from_byte_slices(parts)
