"""CanonicalVote sign-bytes restatement (TEST INFRASTRUCTURE ONLY).

Follows, field for field:
* ``types/block.go:784-810``   Commit.GetVote / Commit.VoteSignBytes
* ``types/block.go:652-665``   CommitSig.BlockID (flag -> BlockID; unknown flag panics)
* ``types/vote.go:93-101``     VoteSignBytes = protoio.MarshalDelimited(CanonicalizeVote)
* ``types/canonical.go:18-34,56-65``  CanonicalizeBlockID (zero BlockID -> nil) / CanonicalizeVote
* ``proto/tendermint/types/canonical.pb.go:370-428,517-579``  gogoproto field order, zero-field
  omission, varint encoding
* ``libs/protoio/writer.go:54-100``  uvarint length prefix
* gogoproto v1.3.2 ``StdTimeMarshalTo`` (external): Timestamp{1: seconds int64 varint,
  2: nanos int32 varint}, zero fields omitted.

Pinned by the five byte-exact vectors of ``types/vote_test.go:60-137``.
"""
from __future__ import annotations

import struct

PREVOTE_TYPE = 1
PRECOMMIT_TYPE = 2

# Go's zero time.Time: Unix() == -62135596800, nanos 0 (vote_test.go:70).
ZERO_TIME = (-62135596800, 0)


def uvarint(v: int) -> bytes:
    v &= (1 << 64) - 1  # Go converts int64 -> uint64 (two's complement)
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _field_bytes(tag: int, payload: bytes) -> bytes:
    return bytes([tag]) + uvarint(len(payload)) + payload


def _validate_hash(h: bytes):
    # types/validation.go ValidateHash: len 0 or tmhash.Size (32)
    if len(h) not in (0, 32):
        raise ValueError("expected size to be 32 bytes, got %d bytes" % len(h))


def canonical_block_id(hash_: bytes, psh_total: int, psh_hash: bytes):
    """``CanonicalizeBlockID``: returns the encoded CanonicalBlockID body, or None for a zero BlockID."""
    _validate_hash(hash_)
    _validate_hash(psh_hash)
    if len(hash_) == 0 and psh_total == 0 and len(psh_hash) == 0:
        return None
    psh = b""
    if psh_total != 0:
        psh += b"\x08" + uvarint(psh_total)
    if len(psh_hash) > 0:
        psh += _field_bytes(0x12, psh_hash)
    body = b""
    if len(hash_) > 0:
        body += _field_bytes(0x0A, hash_)
    body += _field_bytes(0x12, psh)  # PartSetHeader is non-nullable: always emitted
    return body


def timestamp_body(seconds: int, nanos: int) -> bytes:
    out = b""
    if seconds != 0:
        out += b"\x08" + uvarint(seconds)
    if nanos != 0:
        out += b"\x10" + uvarint(nanos)
    return out


def vote_sign_bytes(chain_id: str, type_: int, height: int, round_: int,
                    block_id, timestamp) -> bytes:
    """``VoteSignBytes(chainID, vote)``.

    ``block_id`` is ``(hash, psh_total, psh_hash)`` or None; ``timestamp`` is ``(seconds, nanos)``.
    """
    body = b""
    if type_ != 0:
        body += b"\x08" + uvarint(type_)
    if height != 0:
        body += b"\x11" + struct.pack("<q", height)
    if round_ != 0:
        body += b"\x19" + struct.pack("<q", round_)
    if block_id is not None:
        cbid = canonical_block_id(*block_id)
        if cbid is not None:
            body += _field_bytes(0x22, cbid)
    body += _field_bytes(0x2A, timestamp_body(*timestamp))
    cid = chain_id.encode()
    if cid:
        body += _field_bytes(0x32, cid)
    return uvarint(len(body)) + body
