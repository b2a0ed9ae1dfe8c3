"""Host code under the sanitizers (CPU only; the GPU pool refuses device sanitizers, so these
cover the host side the seam runs on its threads).  tests/native/keycache_fuzz.cpp drives the
key-set cache policy (csrc/keycache.h) through randomized overlapping calls — pins, fast-path hits,
lookups with stale set hashes, deferred and failing builds, budget and LRU changes — under
AddressSanitizer + UndefinedBehaviorSanitizer, checking that every index a call holds names its
own key in the pool until the call ends.  tests/native/pool_stress.cpp runs the seam's host
worker pool (csrc/host_pool.h) from several caller threads with nested calls and throwing parts
under ThreadSanitizer.  Either binary exits non-zero on a broken invariant; a sanitizer report
aborts it."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "tendermint-fork_amd", "csrc")
NATIVE = os.path.join(HERE, "native")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")


def _build(tmp_path, src, flags):
    exe = str(tmp_path / os.path.splitext(src)[0])
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", *flags, "-I", CSRC, os.path.join(NATIVE, src), "-o", exe,
                    "-lpthread"], check=True, capture_output=True, timeout=300)
    return exe


def _run(cmd, env=None):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_keycache_policy_fuzz_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "keycache_fuzz.cpp", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    for seed in (11, 12):
        out = _run([exe, str(seed), "100000"], env)
        assert "failures 0" in out, out


def test_host_pool_stress_tsan(tmp_path):
    exe = _build(tmp_path, "pool_stress.cpp", ["-fsanitize=thread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    out = _run([exe, "4", "10000"], env)
    assert "0 bad" in out, out
