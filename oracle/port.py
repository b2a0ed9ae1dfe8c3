"""ctypes binding to ``oracle/ed25519_port.c`` (TEST INFRASTRUCTURE ONLY).

The C restatement of the Go 1.18 verify rule: used by tests as the checker at
sizes the big-int oracle cannot reach, and by ``bench.py``'s cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libed25519_port.so")
_lib = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        l = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        l.port_verify.restype = ctypes.c_int
        l.port_verify.argtypes = [P, P, ctypes.c_size_t, P, ctypes.c_size_t]
        l.port_verify_batch.restype = None
        l.port_verify_batch.argtypes = [P, P, P, P, P, ctypes.c_size_t, P, ctypes.c_int]
        l.port_verify_batch_zip215.restype = None
        l.port_verify_batch_zip215.argtypes = [P, P, P, P, P, ctypes.c_size_t, P, ctypes.c_int]
        l.port_verify_zip215.restype = ctypes.c_int
        l.port_verify_zip215.argtypes = [P, P, ctypes.c_size_t, P, ctypes.c_size_t]
        l.port_sign_batch.restype = None
        l.port_sign_batch.argtypes = [P, P, P, ctypes.c_size_t, P, P, ctypes.c_int]
        l.port_sign.argtypes = [P, P, ctypes.c_size_t, P]
        l.port_pubkey_from_seed.argtypes = [P, P]
        l.port_sha512.argtypes = [P, ctypes.c_size_t, P]
        l.port_sc_reduce64.argtypes = [P, P]
        _lib = l
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    return bool(lib().port_verify(pub, msg, len(msg), sig, len(sig)))


def sign(seed: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().port_sign(seed, msg, len(msg), out)
    return out.raw


def pubkey_from_seed(seed: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().port_pubkey_from_seed(seed, out)
    return out.raw


def verify_zip215(pub: bytes, msg: bytes, sig: bytes) -> bool:
    """The opt-in ZIP-215 rule (port_verify_zip215; parity with the reference unpinned)."""
    return bool(lib().port_verify_zip215(pub, msg, len(msg), sig, len(sig)))


def verify_batch(pubs: np.ndarray, sigs: np.ndarray, msgs: np.ndarray, offs: np.ndarray,
                 nthreads: int = 1, siglens: np.ndarray | None = None, zip215: bool = False) -> np.ndarray:
    """pubs: (n,32) u8, sigs: (n,64) u8, msgs: flat u8, offs: (n+1,) u64 -> (n,) u8.
    zip215: the opt-in cofactored rule (port_verify_batch_zip215) instead of Go 1.18's."""
    n = pubs.shape[0]
    pubs = np.ascontiguousarray(pubs, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    out = np.zeros(n, dtype=np.uint8)
    sl = None if siglens is None else np.ascontiguousarray(siglens, dtype=np.uint32)
    fn = lib().port_verify_batch_zip215 if zip215 else lib().port_verify_batch
    fn(_ptr(pubs), _ptr(sigs), None if sl is None else _ptr(sl), _ptr(msgs), _ptr(offs), n, _ptr(out), nthreads)
    return out


def sign_batch(seeds: np.ndarray, msgs: np.ndarray, offs: np.ndarray, nthreads: int = 1):
    n = seeds.shape[0]
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    sigs = np.zeros((n, 64), dtype=np.uint8)
    pubs = np.zeros((n, 32), dtype=np.uint8)
    lib().port_sign_batch(_ptr(seeds), _ptr(msgs), _ptr(offs), n, _ptr(sigs), _ptr(pubs), nthreads)
    return sigs, pubs


def sha512(m: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().port_sha512(m, len(m), out)
    return out.raw


def openssl_verify_batch(pubs: np.ndarray, sigs: np.ndarray, msgs: np.ndarray, offs: np.ndarray,
                         nthreads: int = 1):
    """OpenSSL 3 EVP_DigestVerify(ED25519) over the batch (oracle/openssl_anchor.c): the independent
    CPU anchor of bench.py's cpu_baseline leg — not the reference semantics.  None when the anchor
    library (OpenSSL 3) is unavailable."""
    path = os.path.join(_HERE, "_build", "libossl_anchor.so")
    try:
        l = ctypes.CDLL(path)
    except OSError:
        return None
    P = ctypes.c_void_p
    l.ossl_verify_batch.restype = None
    l.ossl_verify_batch.argtypes = [P, P, P, P, ctypes.c_size_t, P, ctypes.c_int]
    n = pubs.shape[0]
    pubs = np.ascontiguousarray(pubs, np.uint8)
    sigs = np.ascontiguousarray(sigs, np.uint8)
    msgs = np.ascontiguousarray(msgs, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    out = np.zeros(n, np.uint8)
    l.ossl_verify_batch(_ptr(pubs), _ptr(sigs), _ptr(msgs), _ptr(offs), n, _ptr(out), nthreads)
    return out
