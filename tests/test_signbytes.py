"""Sign-bytes restatement vs the reference's byte vectors (types/vote_test.go:60-137)."""
import json
import os

from oracle.signbytes import ZERO_TIME, vote_sign_bytes

HERE = os.path.dirname(os.path.abspath(__file__))


def _fixture():
    with open(os.path.join(HERE, "golden", "signbytes_vectors.json")) as f:
        return json.load(f)


def test_reference_vote_sign_bytes_vectors():
    # TestVoteSignBytesTestVectors: 5 byte-exact vectors (zero time, no BlockID)
    for v in _fixture()["reference_vectors"]:
        got = vote_sign_bytes(v["chain_id"], v["type"], v["height"], v["round"], None, ZERO_TIME)
        assert got.hex() == v["want"], v


def test_commit_vote_fixtures_roundtrip():
    for v in _fixture()["commit_votes"]:
        bid = None if v["nil"] else (bytes.fromhex(v["hash"]), v["psh_total"], bytes.fromhex(v["psh_hash"]))
        got = vote_sign_bytes(v["chain_id"], 2, v["height"], v["round"], bid, tuple(v["ts"]))
        assert got.hex() == v["want"]


def test_commit_vote_length_structure():
    # complete BlockID, height > 0: the round field costs 9 bytes when non-zero, the
    # chain ID len+2; every such vote (with R||A) hashes in exactly 2 SHA-512 blocks.
    bid = (b"\x11" * 32, 123, b"\x22" * 32)
    ts = (1672531200, 123456789)  # 5-byte seconds varint, 4-byte nanos varint
    a = vote_sign_bytes("test_chain_id", 2, 3, 0, bid, ts)
    b = vote_sign_bytes("test_chain_id", 2, 3, 1, bid, ts)
    assert len(a) == 114 and len(b) == len(a) + 9
    for m in (a, b, vote_sign_bytes("x" * 50, 2, 3, 1, bid, ts)):
        assert 128 < 64 + len(m) + 17 <= 256
