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
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    assert lib().tmed_device_count() == 0
    with pytest.raises(TmedError):
        Engine(0)
