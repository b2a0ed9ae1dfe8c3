"""The seam's cross-stream ordering under device-side delays: the pipelined seam copies each
batch's staged votes on a copy stream (and signature runs straight from pinned caller memory)
while the kernel lanes run the batch before, and it appends the key-set pool's keys on the
context stream while key-cached batches run on the second lane.  A consumer that does not wait
for its producer's event reads unfinished data only when the producer is late, which the normal
schedule almost never makes it.  Here every batch copy and every key append starts behind a
~200-us sleeping wave on its own stream (tmed_test_stream_delay), and the seam tests whose work
crosses those streams must still equal the oracle loops."""
import ctypes
import time

import numpy as np
import pytest

from conftest import engine_with_env
from tmed._native import lib
from tmed.workload import pubkeys_of, seeds_from_tag
from test_gpu_commit import test_blocksync_pinned_signatures_gpu as _bs_pinned
from test_gpu_commit import test_blocksync_stream_of_windows_gpu as _bs_stream
from test_gpu_commit import test_pipelined_seam_gpu as _pipelined
from test_gpu_configs import test_c3_many_sets_through_the_cache as _c3_many_sets
from test_gpu_configs import test_c4_10k_validator_light_window as _c4_window
from test_gpu_keycache import test_blocksync_window_builds_its_keys_first as _bs_builds_keys
from test_gpu_keycache import test_pool_grows_under_throughput_batches as _pool_grows

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def delay():
    f = lib().tmed_test_stream_delay
    f.argtypes = [ctypes.c_int]
    f.restype = None
    f(200)
    yield
    f(0)


@pytest.fixture
def cache_on():
    e = engine_with_env(TMED_KEYCACHE=1)
    e.keycache_config(True, 16 << 30)
    yield e
    e.close()


def test_delay_hook_is_live(engine):
    """The hook delays what it claims to: a key-set load (its key append behind the sleeping wave,
    then a synchronisation) takes at least the delay longer with 30 ms than with none."""
    f = lib().tmed_test_stream_delay
    pubs = np.asarray(pubkeys_of(engine, seeds_from_tag(b"tmed-delay-live", 0, 8)))

    def load_s(us):
        f(us)
        t0 = time.perf_counter()
        h = engine.keyset_load(pubs)
        dt = time.perf_counter() - t0
        engine.keyset_free(h)
        return dt

    load_s(0)
    fast = min(load_s(0) for _ in range(3))
    slow = load_s(30000)
    f(200)
    assert slow - fast > 0.025, (fast, slow)


def test_c3_many_sets_delayed(engine, cache_on, monkeypatch):
    _c3_many_sets(engine, cache_on, monkeypatch, 40, 2050, "70000")


def test_pipelined_seam_delayed(engine):
    _pipelined(engine)


@pytest.mark.parametrize("keyed", [False, True])
def test_blocksync_stream_delayed(engine, keyed):
    _bs_stream(engine, keyed)


@pytest.mark.parametrize("pinned", ["all", "separate"])
def test_blocksync_pinned_delayed(engine, pinned):
    _bs_pinned(engine, pinned, True)


def test_blocksync_builds_keys_delayed(cache_on, engine):
    _bs_builds_keys(cache_on, engine)


def test_pool_grows_delayed(engine):
    _pool_grows(engine)


def test_c4_window_delayed(engine):
    _c4_window(engine)
