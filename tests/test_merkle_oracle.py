"""Pin the Merkle oracle (oracle/merkle.py) on the reference's own known answers, and check the
kernels' SHA-256 paths (csrc/sha256.h compiled for the host, test-only) against hashlib."""
import ctypes
import hashlib
import random

import pytest

from oracle import merkle as M

# crypto/merkle/tree_test.go:22-44
TREE_KATS = [
    ([], "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    ([b"\x01\x02\x03"], "054edec1d0211f624fed0cbca9d4f9400b0e491c43742af2c5b0abebf0c990d8"),
    ([b""], "6e340b9cffb37a989ca544e6bb780a2c78901d3fb33738768511a30617afa01d"),
    ([b"\x01\x02\x03", b"\x04\x05\x06"], "82e6cfce00453804379b53962939eaa7906b39904be0813fcadd31b100773c4b"),
    ([b"\x01\x02", b"\x03\x04", b"\x05\x06", b"\x07\x08", b"\x09\x0a"],
     "f326493eceab4f2d9ffbc78c59432a0a005d6ea98392045c74df5d14a113be18"),
]


def kat_header():
    """types/block_test.go:311-326 ("Generates expected hash")."""
    s = lambda x: hashlib.sha256(x).digest()
    return {"version_block": 1, "version_app": 2, "chain_id": "chainId", "height": 3,
            "time": (1570983284, 0),                      # 2019-10-13T16:14:44Z
            "last_block_id": (bytes(32), 6, bytes(32)),
            "last_commit_hash": s(b"last_commit_hash"), "data_hash": s(b"data_hash"),
            "validators_hash": s(b"validators_hash"), "next_validators_hash": s(b"next_validators_hash"),
            "consensus_hash": s(b"consensus_hash"), "app_hash": s(b"app_hash"),
            "last_results_hash": s(b"last_results_hash"), "evidence_hash": s(b"evidence_hash"),
            "proposer_address": s(b"proposer_address")[:20]}


KAT_HEADER_HASH = "F740121F553B5418C3EFBD343C2DBFE9E007BB67B0D020A0741374BAB65242A4"


@pytest.mark.parametrize("items,exp", TREE_KATS)
def test_tree_kats(items, exp):
    assert M.hash_from_byte_slices(items).hex() == exp
    assert M.hash_from_byte_slices_iterative(items).hex() == exp


def test_header_hash_kat():
    h = kat_header()
    assert M.header_hash(h).hex().upper() == KAT_HEADER_HASH
    h["validators_hash"] = b""
    assert M.header_hash(h) is None                      # "nil ValidatorsHash yields nil"


def test_empty_valset_hash():
    # types/validator_set_test.go:49-51
    assert M.valset_hash([]).hex() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"


def test_iterative_equals_recursive():
    # tree_test.go:104-116 (TestHashAlternatives), all sizes 0..140
    rng = random.Random(4)
    for n in range(141):
        items = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))) for _ in range(n)]
        assert M.hash_from_byte_slices(items) == M.hash_from_byte_slices_iterative(items)


def test_partset_root_is_tree_of_chunks():
    data = bytes(range(256)) * 5
    assert M.partset_root(data, 100) == M.hash_from_byte_slices([data[i:i + 100] for i in range(0, len(data), 100)])
    assert M.partset_root(b"", 64) == M.empty_hash()


def test_kernel_sha256_paths_hostsim(hostsim):
    """sha256_prefixed (leaf: 0x00 || x, and plain) and sha256_inner vs hashlib, every length
    across the 55/56/64-byte padding boundaries and several 64-byte blocks."""
    rng = random.Random(8)
    out = ctypes.create_string_buffer(32)
    for n in list(range(0, 200)) + [255, 256, 257, 1000, 4095, 4096, 4097]:
        m = bytes(rng.randrange(256) for _ in range(n))
        # offset the buffer so every misalignment is exercised by the word reader
        for shift in (0, 1, 3):
            buf = ctypes.create_string_buffer(bytes(shift) + m + bytes(8))
            ptr = ctypes.cast(ctypes.addressof(buf) + shift, ctypes.c_void_p)
            hostsim.hostsim_sha256(1, 0, ptr, n, out)
            assert out.raw == hashlib.sha256(b"\x00" + m).digest(), (n, shift)
            hostsim.hostsim_sha256(0, 0, ptr, n, out)
            assert out.raw == hashlib.sha256(m).digest(), (n, shift)
    for _ in range(50):
        l, r = rng.randbytes(32), rng.randbytes(32)
        hostsim.hostsim_sha256_inner(l, r, out)
        assert out.raw == M.inner_hash(l, r)
