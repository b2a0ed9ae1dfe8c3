"""Host code under the sanitizers (CPU only; the GPU pool refuses device sanitizers, so these
cover the host side the seam runs on its threads).  tests/native/keycache_fuzz.cpp drives the
key-set cache policy (csrc/keycache.h) through randomized overlapping calls — pins, fast-path hits,
lookups with stale set hashes, deferred and failing builds, budget and LRU changes — under
AddressSanitizer + UndefinedBehaviorSanitizer, checking that every index a call holds names its
own key in the pool until the call ends.  tests/native/pool_stress.cpp runs the seam's host
worker pool (csrc/host_pool.h) from several caller threads with nested calls and throwing parts
under ThreadSanitizer.  tests/native/seam_race.cpp runs the commit seam's host half
(csrc/seam_host.h: planning, the parallel merge, aliasing, staging groups, the part-wise finish)
under ThreadSanitizer with the pool jitter on, and is shown to catch round 5's add_run race.
Either binary exits non-zero on a broken invariant; a sanitizer report aborts it."""
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


SEAM_ARGS = ["600", "48", "3"]  # headers (x2 requests), validators, iterations


def _build_seam(tmp_path, csrc, name, flags):
    """tests/native/seam_race.cpp against the seam's host half in `csrc` (seam_host.h + signbytes.hip)."""
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", *flags, "-I", csrc, os.path.join(NATIVE, "seam_race.cpp"),
                    "-x", "c++", os.path.join(csrc, "signbytes.hip"), "-o", exe, "-lpthread"],
                   check=True, capture_output=True, timeout=300)
    return exe


def _digest(out):
    return out.split("digest")[-1].strip()


def test_seam_host_regions_race_free_tsan(tmp_path):
    """The commit seam's host half as the pipelined seam runs it (seam_plan with a staging group and
    template rows, the part-wise finish) on a light-client batch, under ThreadSanitizer with the pool
    jitter on; its outcomes equal those of one host thread (every region serial)."""
    tsan = _build_seam(tmp_path, CSRC, "seam_race_tsan", ["-fsanitize=thread"])
    plain = _build_seam(tmp_path, CSRC, "seam_race", [])
    serial = _run([plain] + SEAM_ARGS + ["0", "7"], dict(os.environ, TMED_HOST_THREADS="1"))
    for threads, jitter, seed in (("8", "200", "7"), ("5", "50", "7")):
        env = dict(os.environ, TMED_HOST_THREADS=threads, TSAN_OPTIONS="halt_on_error=1")
        out = _run([tsan] + SEAM_ARGS + [jitter, seed], env)
        assert "parts %s " % threads in out and " aliases 0 " not in out, out  # the part-wise finish ran
        assert _digest(out) == _digest(serial), (out, serial)


def test_seam_race_harness_catches_round5_add_run(tmp_path):
    """The harness fails the round-5 seam: Group::add_run ending a run at off[r + 1], which the next
    planning part's worker is still writing (fixed in commit.hip, now seam_host.h), is reported by
    ThreadSanitizer on the first run."""
    old = tmp_path / "csrc"
    shutil.copytree(CSRC, str(old), ignore=shutil.ignore_patterns("*.hip"))
    shutil.copy(os.path.join(CSRC, "signbytes.hip"), str(old))
    inc = os.path.abspath(os.path.join(CSRC, "..", "..", "include", "tmed25519.h"))
    for f in os.listdir(str(old)):
        p = old / f
        s = p.read_text().replace('"../../include/tmed25519.h"', '"%s"' % inc)
        if f == "seam_host.h":
            fixed = "const size_t c0 = c.off[r], c1 = c0 + c.runs[r].len;"
            assert fixed in s
            s = s.replace(fixed, "const size_t c0 = c.off[r], c1 = c.off[r + 1];")
        p.write_text(s)
    exe = _build_seam(tmp_path, str(old), "seam_race_old", ["-fsanitize=thread"])
    env = dict(os.environ, TMED_HOST_THREADS="8", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe] + SEAM_ARGS + ["200", "7"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "data race" in r.stderr and "add_run" in r.stderr, r.stderr[-3000:]
