"""Loader for the gfx950 engine library (libtmed25519_hip.so) — fails loudly.

There is no CPU fallback in the product: if the library is missing, or no
gfx950 device is present, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TMED_LIB overrides the library path (A/B runs of two builds of the same sources).
LIB_PATH = os.environ.get("TMED_LIB") or os.path.join(PKG_ROOT, "lib", "libtmed25519_hip.so")

TMED_OK = 0
TMED_EINVAL = -1
TMED_ENODEV = -2
TMED_EHIP = -3
TMED_ENOMEM = -4
TMED_ENOKEYSET = -5
TMED_EINTERNAL = -6

_lib = None


class TmedError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().tmed_strerror(code).decode() if _lib is not None else str(code)
        super().__init__("%s: %s (code %d)" % (what or "tmed", msg, code))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: when PyTorch-ROCm is present its bundled
    # libamdhip64.so.7 must be the one loaded (our NEEDED libamdhip64.so.7 then
    # binds to it).  Loading ours first would pull /opt/rocm's copy and a second
    # runtime would appear when torch loads, which cannot see the GPUs.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("tmed: %s is missing — run __graft_entry__.build() (hipcc --offload-arch=gfx950); "
                          "there is no CPU fallback" % LIB_PATH)
    l = ctypes.CDLL(LIB_PATH)
    P, SZ, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    l.tmed_device_count.restype = I
    l.tmed_device_count.argtypes = []
    l.tmed_init.restype = I
    l.tmed_init.argtypes = [I, ctypes.POINTER(P)]
    l.tmed_destroy.restype = None
    l.tmed_destroy.argtypes = [P]
    l.tmed_strerror.restype = ctypes.c_char_p
    l.tmed_strerror.argtypes = [I]
    l.tmed_verify_batch.restype = I
    l.tmed_verify_batch.argtypes = [P, P, P, P, P, P, SZ, P]
    l.tmed_verify_batch_device.restype = I
    l.tmed_verify_batch_device.argtypes = [P, P, P, P, P, SZ, P, P]
    l.tmed_sign_batch.restype = I
    l.tmed_sign_batch.argtypes = [P, P, P, P, SZ, P, P]
    l.tmed_sign_batch_device.restype = I
    l.tmed_sign_batch_device.argtypes = [P, P, P, P, SZ, P, P, P]
    l.tmed_keyset_load.restype = I
    l.tmed_keyset_load.argtypes = [P, P, SZ, ctypes.POINTER(ctypes.c_uint64)]
    l.tmed_keyset_free.restype = I
    l.tmed_keyset_free.argtypes = [P, ctypes.c_uint64]
    l.tmed_keyset_extend.restype = I
    l.tmed_keyset_extend.argtypes = [P, ctypes.c_uint64, P, SZ, ctypes.POINTER(ctypes.c_uint32)]
    l.tmed_keycache_config.restype = I
    l.tmed_keycache_config.argtypes = [P, I, SZ]
    l.tmed_keycache_stats.restype = I
    l.tmed_keycache_stats.argtypes = [P, P]
    l.tmed_keycache_wait.restype = I
    l.tmed_keycache_wait.argtypes = [P]
    l.tmed_keycache_flush.restype = I
    l.tmed_keycache_flush.argtypes = [P]
    l.tmed_keycache_warm.restype = I
    l.tmed_keycache_warm.argtypes = [P, P]
    l.tmed_verify_batch_keyset.restype = I
    l.tmed_verify_batch_keyset.argtypes = [P, ctypes.c_uint64, P, P, P, P, P, SZ, P]
    l.tmed_verify_batch_keyset_device.restype = I
    l.tmed_verify_batch_keyset_device.argtypes = [P, ctypes.c_uint64, P, P, P, P, SZ, P, P]
    l.tmed_set_kernel_timing.restype = I
    l.tmed_set_kernel_timing.argtypes = [P, I]
    l.tmed_kernel_times.restype = I
    l.tmed_kernel_times.argtypes = [P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]
    l.tmed_last_kernel_ms.restype = ctypes.c_float
    l.tmed_last_kernel_ms.argtypes = [P]
    l.tmed_window_stats.restype = I
    l.tmed_window_stats.argtypes = [P, P, P]
    l.tmed_b_window_bits.restype = I
    l.tmed_b_window_bits.argtypes = [P]
    l.tmed_keyset_b_window_bits.restype = I
    l.tmed_keyset_b_window_bits.argtypes = [P]
    l.tmed_keyset_a_window_bits.restype = I
    l.tmed_keyset_a_window_bits.argtypes = [P, ctypes.c_uint64]
    l.tmed_keyset_comb_entry.restype = I
    l.tmed_keyset_comb_entry.argtypes = [P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32,
                                         ctypes.c_uint32, P]
    l.tmed_host_alloc.restype = I
    l.tmed_host_alloc.argtypes = [SZ, ctypes.POINTER(ctypes.c_void_p)]
    l.tmed_host_free.restype = I
    l.tmed_host_free.argtypes = [P]
    l.tmed_host_register.restype = I
    l.tmed_host_register.argtypes = [P, SZ]
    l.tmed_host_unregister.restype = I
    l.tmed_host_unregister.argtypes = [P]
    l.tmed_verify_batch_zip215.argtypes = [P, P, P, P, P, P, SZ, P]
    l.tmed_verify_batch_zip215_device.argtypes = [P, P, P, P, P, SZ, P, P]
    l.tmed_zip215_set_seed.argtypes = [P]
    l.tmed_zip215_stats.argtypes = [P]
    l.tmed_test_pool_jitter.restype = None
    l.tmed_test_pool_jitter.argtypes = [I]
    l.tmed_test_stream_delay.restype = None
    l.tmed_test_stream_delay.argtypes = [I]
    l.tmed_debug_zero_bits.restype = I
    l.tmed_debug_zero_bits.argtypes = [P, SZ, ctypes.POINTER(SZ)]
    _lib = l
    return l


# Every symbol include/tmed25519.h declares (checked by the CPU test suite).
EXPORTED_SYMBOLS = [
    "tmed_device_count", "tmed_init", "tmed_destroy", "tmed_strerror",
    "tmed_verify_batch", "tmed_verify_batch_device",
    "tmed_sign_batch", "tmed_sign_batch_device", "tmed_last_kernel_ms",
    "tmed_vote_sign_bytes", "tmed_valu_peak", "tmed_verify_commits", "tmed_verify_commits_with",
    "tmed_test_pool_jitter", "tmed_test_stream_delay", "tmed_debug_zero_bits",
    "tmed_keyset_load", "tmed_keyset_free", "tmed_keyset_extend", "tmed_verify_batch_keyset",
    "tmed_keycache_config", "tmed_keycache_stats", "tmed_keycache_flush", "tmed_keycache_warm", "tmed_keycache_wait", "tmed_verify_batch_keyset_device",
    "tmed_set_kernel_timing", "tmed_kernel_times", "tmed_blocksync_verify", "tmed_blocksync_submit", "tmed_blocksync_wait",
    "tmed_merkle_roots", "tmed_valset_hashes", "tmed_header_hashes", "tmed_partset_roots",
    "tmed_verify_commits_multi", "tmed_blocksync_verify_multi", "tmed_window_stats", "tmed_b_window_bits", "tmed_keyset_b_window_bits", "tmed_keyset_a_window_bits", "tmed_keyset_comb_entry", "tmed_seam_phase_us",
    "tmed_verify_batch_zip215", "tmed_verify_batch_zip215_device", "tmed_zip215_set_seed", "tmed_zip215_stats",
    "tmed_host_alloc", "tmed_host_free", "tmed_host_register", "tmed_host_unregister",
]
