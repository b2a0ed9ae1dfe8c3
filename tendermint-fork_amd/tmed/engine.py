"""Host-side handle on one GPU: batch verify / sign through the C ABI.

Mirrors the per-signature contract of ``ed25519.PubKey.VerifySignature``
(reference ``crypto/ed25519/ed25519.go:148-155``) for whole batches: each
output byte is exactly the bool the reference would return.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from ._native import TMED_OK, TmedError, lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def pack_messages(msgs: Sequence[bytes]):
    """Concatenate messages -> (flat u8 array, u32 offsets[n+1])."""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.int64, count=len(msgs))
    off = np.zeros(len(msgs) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    if off[-1] >= 2**32:
        raise ValueError("message batch exceeds 4 GiB")
    flat = np.frombuffer(b"".join(msgs), dtype=np.uint8) if off[-1] else np.zeros(1, np.uint8)
    return flat, off.astype(np.uint32)


class PinnedBuffer:
    """Page-locked host memory from tmed_host_alloc: commit arrays marshalled into it reach the
    device by direct DMA in large seam batches (include/tmed25519.h).  Arrays from array() are
    views: keep the buffer alive while they are used, free() it after."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        rc = lib().tmed_host_alloc(int(nbytes), ctypes.byref(p))
        if rc != TMED_OK:
            raise TmedError(rc)
        self.ptr, self.nbytes = p.value, int(nbytes)

    def array(self, shape, dtype, offset: int = 0) -> np.ndarray:
        count = int(np.prod(shape))
        if offset + count * np.dtype(dtype).itemsize > self.nbytes:
            raise ValueError("view past the pinned buffer")
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        return np.frombuffer(raw, dtype, count=count, offset=offset).reshape(shape)

    def free(self) -> None:
        if self.ptr:
            rc = lib().tmed_host_free(self.ptr)
            self.ptr = None
            if rc != TMED_OK:
                raise TmedError(rc)


class Engine:
    """One context on one HIP device (one process per GPU)."""

    def __init__(self, device: int = 0):
        l = lib()
        if l.tmed_device_count() <= device:
            raise TmedError(-2, "tmed_init(device=%d)" % device)
        h = ctypes.c_void_p()
        rc = l.tmed_init(device, ctypes.byref(h))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_init(device=%d)" % device)
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().tmed_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- host buffers -------------------------------------------------------
    def verify_arrays(self, pubs: np.ndarray, sigs: np.ndarray, msgs: np.ndarray, offs: np.ndarray,
                      sig_lens: np.ndarray | None = None) -> np.ndarray:
        n = pubs.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return out
        pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(n, 32)
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(n, 64)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        sl = None if sig_lens is None else np.ascontiguousarray(sig_lens, dtype=np.uint32)
        rc = lib().tmed_verify_batch(self._h, _p(pubs), _p(sigs), None if sl is None else _p(sl), _p(msgs),
                                     _p(offs), n, _p(out))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_batch")
        return out

    def verify_zip215_arrays(self, pubs: np.ndarray, sigs: np.ndarray, msgs: np.ndarray, offs: np.ndarray,
                             sig_lens: np.ndarray | None = None) -> np.ndarray:
        """The opt-in ZIP-215 rule (tmed_verify_batch_zip215): randomized batch equation by MSM,
        bisection, exact single-signature fallback — decisions equal the ZIP-215 single check."""
        n = pubs.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return out
        pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(n, 32)
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(n, 64)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        sl = None if sig_lens is None else np.ascontiguousarray(sig_lens, dtype=np.uint32)
        rc = lib().tmed_verify_batch_zip215(self._h, _p(pubs), _p(sigs), None if sl is None else _p(sl), _p(msgs),
                                            _p(offs), n, _p(out))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_batch_zip215")
        return out

    def verify_zip215_device(self, d_pub, d_sig, d_msg, d_off, d_out, n: int, stream=None) -> None:
        s = ctypes.c_void_p(stream) if stream else None
        rc = lib().tmed_verify_batch_zip215_device(self._h, d_pub.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                                   d_off.data_ptr(), n, d_out.data_ptr(), s)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_batch_zip215_device")

    @staticmethod
    def zip215_set_seed(seed: bytes | None) -> None:
        """Tests only: fixed batch-weight seed for this thread (None: getrandom per call)."""
        rc = lib().tmed_zip215_set_seed(None if seed is None else ctypes.c_char_p(bytes(seed)))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_zip215_set_seed")

    @staticmethod
    def zip215_stats() -> dict:
        out = (ctypes.c_uint32 * 4)()
        rc = lib().tmed_zip215_stats(out)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_zip215_stats")
        return {"chunks": out[0], "equations": out[1], "single_groups": out[2], "single_sigs": out[3]}

    def verify_batch(self, pubs: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> np.ndarray:
        """Decisions for (pub[i], msg[i], sig[i]); sigs of any length (len != 64 -> 0)."""
        n = len(pubs)
        pa = np.zeros((n, 32), np.uint8)
        sa = np.zeros((n, 64), np.uint8)
        sl = np.zeros(n, np.uint32)
        for i in range(n):
            if len(pubs[i]) != 32:
                raise ValueError("ed25519: bad public key length %d" % len(pubs[i]))  # Go panics here
            pa[i] = np.frombuffer(pubs[i], np.uint8)
            s = sigs[i][:64]
            sa[i, :len(s)] = np.frombuffer(s, np.uint8) if s else 0
            sl[i] = len(sigs[i])
        flat, off = pack_messages(list(msgs))
        return self.verify_arrays(pa, sa, flat, off, sl)

    def sign_arrays(self, seeds: np.ndarray, msgs: np.ndarray, offs: np.ndarray):
        n = seeds.shape[0]
        sigs = np.zeros((n, 64), np.uint8)
        pubs = np.zeros((n, 32), np.uint8)
        if n == 0:
            return sigs, pubs
        seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        rc = lib().tmed_sign_batch(self._h, _p(seeds), _p(msgs), _p(offs), n, _p(sigs), _p(pubs))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_sign_batch")
        return sigs, pubs

    # ---- device-resident (torch tensors on this device) ----------------------
    def verify_device(self, d_pub, d_sig, d_msg, d_off, d_out, n: int, stream=None) -> None:
        s = ctypes.c_void_p(stream) if stream else None
        rc = lib().tmed_verify_batch_device(self._h, d_pub.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(),
                                            d_off.data_ptr(), n, d_out.data_ptr(), s)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_batch_device")

    def sign_device(self, d_seed, d_msg, d_off, d_sig_out, d_pub_out, n: int, stream=None) -> None:
        s = ctypes.c_void_p(stream) if stream else None
        rc = lib().tmed_sign_batch_device(self._h, d_seed.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), n,
                                          d_sig_out.data_ptr(), d_pub_out.data_ptr(), s)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_sign_batch_device")

    # ---- key-set cache (per validator set) ----------------------------------
    def keyset_load(self, pubs: np.ndarray) -> int:
        pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(-1, 32)
        h = ctypes.c_uint64(0)
        rc = lib().tmed_keyset_load(self._h, _p(pubs), pubs.shape[0], ctypes.byref(h))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keyset_load")
        return h.value

    def keyset_free(self, handle: int) -> None:
        rc = lib().tmed_keyset_free(self._h, handle)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keyset_free")

    def keyset_extend(self, handle: int, pubs: np.ndarray) -> int:
        """Append keys to a key set (tmed_keyset_extend); returns the first new key's index."""
        pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(-1, 32)
        first = ctypes.c_uint32(0)
        rc = lib().tmed_keyset_extend(self._h, handle, _p(pubs), pubs.shape[0], ctypes.byref(first))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keyset_extend")
        return first.value

    # ---- the commit seam's key-set cache (tmed_keycache_*) -------------------
    KEYCACHE_FIELDS = ("enabled", "budget_bytes", "lookups", "hits", "keyed_sets", "generic_sets", "keyed_sigs",
                       "generic_sigs", "keys_appended", "keys_deferred", "pool_resets", "sets_evicted", "pool_keys",
                       "pool_capacity_keys", "pool_bytes", "pool_a_window_bits", "sets_cached", "pending_keys")

    def keycache_config(self, enabled: bool | None = None, budget_bytes: int = 0) -> None:
        en = -1 if enabled is None else (1 if enabled else 0)
        rc = lib().tmed_keycache_config(self._h, en, int(budget_bytes))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keycache_config")

    def keycache_stats(self) -> dict:
        out = (ctypes.c_uint64 * len(self.KEYCACHE_FIELDS))()
        rc = lib().tmed_keycache_stats(self._h, out)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keycache_stats")
        return {k: int(out[i]) for i, k in enumerate(self.KEYCACHE_FIELDS)}

    def keycache_wait(self) -> None:
        """Block until the keys queued by generic calls are built (tmed_keycache_wait)."""
        rc = lib().tmed_keycache_wait(self._h)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keycache_wait")

    def keycache_flush(self) -> None:
        rc = lib().tmed_keycache_flush(self._h)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keycache_flush")

    def keycache_warm(self, vals) -> None:
        """Build a ValidatorSet's missing keys into the cache now (tmed_keycache_warm)."""
        from .types import _valset_c
        keep = []
        vs = _valset_c(vals, keep)
        rc = lib().tmed_keycache_warm(self._h, ctypes.byref(vs))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_keycache_warm")

    def verify_keyset_arrays(self, handle: int, val_idx: np.ndarray, sigs: np.ndarray, msgs: np.ndarray,
                             offs: np.ndarray, sig_lens: np.ndarray | None = None) -> np.ndarray:
        n = val_idx.shape[0]
        out = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return out
        vi = np.ascontiguousarray(val_idx, dtype=np.uint32)
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(n, 64)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint32)
        sl = None if sig_lens is None else np.ascontiguousarray(sig_lens, dtype=np.uint32)
        rc = lib().tmed_verify_batch_keyset(self._h, handle, _p(vi), _p(sigs), None if sl is None else _p(sl),
                                            _p(msgs), _p(offs), n, _p(out))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_batch_keyset")
        return out

    def verify_keyset_device(self, handle: int, d_val_idx, d_sig, d_msg, d_off, d_out, n: int, stream=None) -> None:
        s = ctypes.c_void_p(stream) if stream else None
        rc = lib().tmed_verify_batch_keyset_device(self._h, handle, d_val_idx.data_ptr(), d_sig.data_ptr(),
                                                   d_msg.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), s)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_verify_batch_keyset_device")

    def set_kernel_timing(self, on: bool) -> None:
        rc = lib().tmed_set_kernel_timing(self._h, 1 if on else 0)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_set_kernel_timing")

    def kernel_times(self):
        """Per kernel kind (prep, main, finish) of the last verify_device call (timing on):
        ([ms...], [launches...])."""
        ms, n = (ctypes.c_float * 3)(), (ctypes.c_int * 3)()
        rc = lib().tmed_kernel_times(self._h, ms, n)
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_kernel_times")
        return list(ms), list(n)

    def window_stats(self):
        """(lane_hist, wave_hist): window counts W of the last half-size chunk (tmed_window_stats)."""
        lh, wh = np.zeros(65, np.uint32), np.zeros(65, np.uint32)
        rc = lib().tmed_window_stats(self._h, _p(lh), _p(wh))
        if rc != TMED_OK:
            raise TmedError(rc, "tmed_window_stats")
        return lh, wh

    def b_window_bits(self) -> int:
        """Radix (bits) of the default path's fixed-base B windows: 26 or 16 (tmed_b_window_bits)."""
        return int(lib().tmed_b_window_bits(self._h))

    def keyset_b_window_bits(self) -> int:
        """Radix (bits) of the key-cached throughput path's B windows: 24 or 16 (tmed_keyset_b_window_bits)."""
        return int(lib().tmed_keyset_b_window_bits(self._h))

    def keyset_a_window_bits(self, handle: int) -> int:
        """Radix (bits) of the -A comb the throughput kernel reads for a key set: 12 or 8
        (tmed_keyset_a_window_bits; 12 once the set's first throughput batch built it)."""
        return int(lib().tmed_keyset_a_window_bits(self._h, handle))

    def keyset_comb_entry(self, handle: int, key: int, radix_bits: int, window: int, j: int) -> np.ndarray:
        """Diagnostic: one comb row of a key set as its 30 int32 limbs (y + x, y - x, 2d x y of
        j * R^window * (-A); tmed_keyset_comb_entry)."""
        out = np.zeros(30, np.int32)
        rc = lib().tmed_keyset_comb_entry(self._h, handle, key, radix_bits, window, j, out.ctypes.data)
        if rc != 0:
            raise TmedError(rc, "tmed_keyset_comb_entry")
        return out

    def last_kernel_ms(self) -> float:
        return float(lib().tmed_last_kernel_ms(self._h))
