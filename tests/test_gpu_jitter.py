"""The seam's host-parallel phases under scheduling jitter: the commit seam plans, merges, stages,
scatters and replays a batch in parts on the host pool (csrc/host_pool.h), and a part that reads
what another part of the same region writes is a race that the normal schedule almost never
shows (round 5 found one: Group::add_run read the next part's first run offset; a false reject
about once in 250 light-client calls, profiles/r05/s28/).  Here every part of every region starts
after a pseudo-random delay of up to 400 us (tmed_test_pool_jitter), and the seam tests whose
batches run in parts — light-client batches with aliased Trusting/Light pairs, pipelined and not,
through the key-set cache and not; blocksync windows and streams; concurrent callers — must still
equal the oracle loops."""
import ctypes

import pytest

from conftest import engine_with_env
from tmed._native import lib
from test_gpu_commit import test_blocksync_stream_of_windows_gpu as _bs_stream
from test_gpu_commit import test_blocksync_window_matches_light_loops as _bs_window
from test_gpu_commit import test_pipelined_seam_gpu as _pipelined
from test_gpu_concurrency import test_concurrent_callers_share_one_context as _concurrent
from test_gpu_configs import test_c3_light_client_changing_sets as _c3_changing
from test_gpu_configs import test_c3_many_sets_through_the_cache as _c3_many_sets
from test_gpu_configs import test_c4_10k_validator_light_window as _c4_window
from test_gpu_keycache import test_c3_changing_sets_without_handles as _c3_no_handles

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def jitter():
    f = lib().tmed_test_pool_jitter
    f.argtypes = [ctypes.c_int]
    f.restype = None
    f(400)
    yield
    f(0)


@pytest.fixture
def cache_on():
    e = engine_with_env(TMED_KEYCACHE=1)
    e.keycache_config(True, 16 << 30)
    yield e
    e.close()


@pytest.mark.parametrize("nv,H,pipe", [(8, 2050, None), (40, 2050, "70000")])
def test_c3_many_sets_jittered(engine, cache_on, monkeypatch, nv, H, pipe):
    _c3_many_sets(engine, cache_on, monkeypatch, nv, H, pipe)


@pytest.mark.parametrize("keyed,pipelined", [(True, True), (False, True), (False, False)])
def test_c3_changing_sets_jittered(engine, monkeypatch, keyed, pipelined):
    _c3_changing(engine, monkeypatch, keyed, pipelined)


def test_c3_without_handles_jittered(cache_on):
    _c3_no_handles(cache_on)


def test_pipelined_seam_jittered(engine):
    _pipelined(engine)


@pytest.mark.parametrize("keyed", [False, True])
def test_blocksync_window_jittered(engine, keyed):
    _bs_window(engine, 3, "bs-chain", keyed)


@pytest.mark.parametrize("keyed", [False, True])
def test_blocksync_stream_jittered(engine, keyed):
    _bs_stream(engine, keyed)


def test_c4_window_jittered(engine):
    _c4_window(engine)


def test_concurrent_callers_jittered(engine):
    _concurrent(engine)
