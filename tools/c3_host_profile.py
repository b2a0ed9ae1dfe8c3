"""Host-side profile of the commit seam on the C3 request shape, CPU only.

Builds the light-client batch of bench_commits.py c3 (headers x 175 validators, one key
replaced per height, Trusting 1/3 + Light per header) with random keys and signatures, and
runs it through tmed_verify_commits_with with a verifier that accepts everything, so the
seam's host phases (plan, replay) are timed without a GPU.  Run with TMED_TRACE=1 for the
per-phase breakdown of the planner.

    TMED_TRACE=1 python tools/c3_host_profile.py --headers 3000
"""
import argparse
import os
import sys
import time

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "tendermint-fork_amd")]


class FakeEngine:
    """sign_arrays stand-in: random public keys and signatures (the verifier ignores them)."""

    def __init__(self):
        self.rng = np.random.default_rng(7)

    def sign_arrays(self, seeds, flat, offs):
        n = seeds.shape[0]
        return (self.rng.integers(0, 256, (n, 64), dtype=np.uint8), self.rng.integers(0, 256, (n, 32), dtype=np.uint8))

    def keyset_load(self, pubs):
        return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--headers", type=int, default=3000)
    ap.add_argument("--gap", type=int, default=2)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--only", choices=["trusting", "light"], default=None, help="one of the two requests per header")
    a = ap.parse_args()
    import bench_commits as bc
    import tmed.types as T
    sets, commits, _, _ = bc._c3_world(FakeEngine(), a.headers, a.gap, False)
    reqs = []
    for h in range(a.headers):
        u = h + a.gap
        if a.only != "light":
            reqs.append((T.MODE_LIGHT_TRUSTING, sets[h], "test_chain_id", None, 0, commits[u], 1, 3))
        if a.only != "trusting":
            reqs.append((T.MODE_LIGHT, sets[u], "test_chain_id", commits[u].block_id, u + 1, commits[u], 0, 0))
    ok = lambda pubs, sigs, lens, msgs, offs: np.ones(pubs.shape[0], np.uint8)
    for r in range(a.runs):
        t0 = time.perf_counter()
        errs = T.verify_commits(None, reqs, verifier=ok)
        dt = time.perf_counter() - t0
        ph = T.seam_phase_us()
        print("run %d: %.1f ms total, plan %.2f ms, verify %.2f ms, replay %.2f ms, errors %d"
              % (r, dt * 1e3, ph[0] / 1e3, ph[1] / 1e3, ph[2] / 1e3, sum(e is not None for e in errs)))


if __name__ == "__main__":
    main()
