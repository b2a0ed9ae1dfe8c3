"""Probe (GPU box): wall time of hipMalloc / hipFree / device-to-device copy at the key pool's
sizes (6.3 MB per key: 10k keys = 63 GB, 20k = 127 GB), to see what a pool growth costs."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipDeviceSynchronize.argtypes = []
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
out = {}


def t(f):
    t0 = time.perf_counter()
    rc = f()
    hip.hipDeviceSynchronize()
    return rc, round(time.perf_counter() - t0, 4)


GB = 1 << 30
a, b = ctypes.c_void_p(), ctypes.c_void_p()
out["malloc_63GB"] = t(lambda: hip.hipMalloc(ctypes.byref(a), 63 * GB))
out["memset_63GB"] = t(lambda: hip.hipMemset(a, 0, 63 * GB))
out["malloc_127GB"] = t(lambda: hip.hipMalloc(ctypes.byref(b), 127 * GB))
out["copy_63GB_d2d"] = t(lambda: hip.hipMemcpy(b, a, 63 * GB, 3))
out["free_63GB"] = t(lambda: hip.hipFree(a))
out["free_127GB"] = t(lambda: hip.hipFree(b))
out["malloc_63GB_again"] = t(lambda: hip.hipMalloc(ctypes.byref(a), 63 * GB))
out["free_63GB_again"] = t(lambda: hip.hipFree(a))
print(json.dumps(out))
