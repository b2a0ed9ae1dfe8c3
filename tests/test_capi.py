"""C-ABI library: loads, exports every symbol include/tmed25519.h declares, and
fails loudly (no CPU fallback) when no gfx950 device is present."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "tmed25519.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|float|const char \*)\s*\*?\s*(tmed_\w+)\s*\(", src, re.M)))


def test_library_exports_header_symbols():
    from tmed import _native
    if not os.path.exists(_native.LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tendermint-fork_amd")])
    out = subprocess.check_output(["nm", "-D", "--defined-only", _native.LIB_PATH]).decode()
    exported = set(re.findall(r"\bT (tmed_\w+)", out))
    declared = _declared_symbols()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert set(_native.EXPORTED_SYMBOLS) == set(declared)
    l = _native.lib()
    for s in declared:
        assert hasattr(l, s)


def test_strerror_and_no_fallback_without_gpu():
    import torch
    from tmed import Engine, TmedError, lib
    assert lib().tmed_strerror(-2).decode().startswith("no usable")
    # a host-side exception is its own code, never reported as a HIP (device) error
    from tmed import _native
    assert lib().tmed_strerror(_native.TMED_EINTERNAL).decode().startswith("internal error")
    assert lib().tmed_strerror(_native.TMED_EHIP).decode() == "HIP runtime error"
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    assert lib().tmed_device_count() == 0
    with pytest.raises(TmedError):
        Engine(0)


def test_pinned_memory_entry_points_reject_bad_arguments():
    """tmed_host_alloc / _free / _register / _unregister (the pinned commit arenas the seam DMAs
    signatures from): argument errors come back as TMED_EINVAL without touching the runtime, and a
    pointer the registry never saw cannot be freed or unregistered."""
    import ctypes
    from tmed import lib
    l = lib()
    p = ctypes.c_void_p()
    assert l.tmed_host_alloc(0, ctypes.byref(p)) == -1
    assert l.tmed_host_alloc(16, None) == -1
    assert l.tmed_host_free(None) == 0          # free(NULL) is a no-op
    buf = ctypes.create_string_buffer(64)
    assert l.tmed_host_free(ctypes.addressof(buf)) == -1
    assert l.tmed_host_unregister(None) == -1
    assert l.tmed_host_unregister(ctypes.addressof(buf)) == -1
    assert l.tmed_host_register(None, 64) == -1
    assert l.tmed_host_register(ctypes.addressof(buf), 0) == -1
