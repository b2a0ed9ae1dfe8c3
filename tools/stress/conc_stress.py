"""Diagnostic (round 5): the two concurrent-caller tests — tests/test_gpu_concurrency.py (every entry
point of one cache-off context from seven threads, device-pointer batches on their own streams) and
tests/test_gpu_product_default.py::test_concurrent_callers_cache_on (blocksync windows, single
commits on sets changing every three calls while the key-cache worker builds, a light client) —
repeated on fresh contexts, each run checked against the port / the oracle loops as in the tests.
Usage: python tools/stress/conc_stress.py [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, ROOT)

from conftest import engine_with_env  # noqa: E402
from test_gpu_concurrency import test_concurrent_callers_share_one_context as shared  # noqa: E402
from test_gpu_product_default import _cache_on, test_concurrent_callers_cache_on as cache_on  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    fails, t0 = 0, time.perf_counter()
    for r in range(rounds):
        for name, make, fn in (("shared", lambda: engine_with_env(), shared), ("cache_on", _cache_on, cache_on)):
            e = make()
            try:
                fn(e)
            except AssertionError as ex:
                fails += 1
                print("round %d %s FAILED: %s" % (r, name, str(ex)[:400]), flush=True)
            finally:
                e.close()
        print("round %d done, %d failures, %.1f s" % (r, fails, time.perf_counter() - t0), flush=True)
    print("total failures", fails, flush=True)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
