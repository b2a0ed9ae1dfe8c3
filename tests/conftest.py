import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tendermint-fork_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


# the test suite fixes ZIP-215 batch weights (tmed_zip215_set_seed refuses otherwise)
os.environ.setdefault("TMED_ZIP215_TEST_SEED", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def hostsim():
    """TEST-ONLY CPU build of the kernel source (tests/native/hostsim.cpp)."""
    import ctypes
    d = os.path.join(ROOT, "tests", "native")
    subprocess.check_call(["make", "-s", "-C", d])
    return ctypes.CDLL(os.path.join(d, "libhostsim.so"))


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "ed25519_vectors.json")) as f:
        return json.load(f)["vectors"]


@pytest.fixture(scope="session")
def engine():
    """The shared test context, with the seam's key-set cache OFF: a set without a handle takes the
    generic kernels on every call, so each test exercises the path it names (the cache itself is
    tested on its own contexts: tests/test_gpu_keycache.py)."""
    from tmed import Engine
    e = Engine(0)
    e.keycache_config(False)
    yield e
    e.close()


def engine_with_env(**env):
    """A second context created with TMED_* overrides (read by tmed_init only); the key-set cache
    is off unless TMED_KEYCACHE is given."""
    from tmed import Engine
    env.setdefault("TMED_KEYCACHE", 0)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return Engine(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="session")
def generic_engines():
    """The generic path's two kernel pipelines on the same inputs: the latency kernels
    (latency.hip, every batch up to kGLatMax) and the throughput kernels (TMED_GLAT_MAX=0)."""
    es = {"latency": engine_with_env(TMED_GLAT_MAX=1 << 16), "throughput": engine_with_env(TMED_GLAT_MAX=0)}
    yield es
    for e in es.values():
        e.close()


@pytest.fixture(params=["latency", "throughput"])
def generic_engine(request, generic_engines):
    return generic_engines[request.param]
