"""Diagnostic (round 5): random commit scenarios (tests/commit_cases.py: 1-31 validators, every
flag, wrong BlockIDs / heights, double votes, bad signatures before and after the crossings, three
chain IDs, the three loops) through tmed_verify_commits on a cache-off and a cache-on context, for
many seeds, against the oracle loops.  Usage: python tools/stress/commit_stress.py [seeds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, ROOT)

from commit_cases import oracle_outcome, pbid, same_outcome, scenarios  # noqa: E402
from conftest import engine_with_env  # noqa: E402
import tmed.types as T  # noqa: E402


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    off = engine_with_env()
    on = engine_with_env(TMED_KEYCACHE=1)
    on.keycache_config(True, 8 << 30)
    bad, t0, total = 0, time.perf_counter(), 0
    for sd in range(1000, 1000 + seeds):
        reqs, exp = [], []
        for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=sd, count=60):
            exp.append(oracle_outcome(mode, vs, chain, bid, h, cm, num, den))
            reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
        for name, e in (("off", off), ("on", on), ("on", on)):  # the cache-on context twice: cold, then warm
            got = T.verify_commits(e, reqs)
            if name == "on":
                e.keycache_wait()
            miss = [(q, str(g)[:60], str(x)[:60]) for q, (g, x) in enumerate(zip(got, exp)) if not same_outcome(g, x)]
            total += len(reqs)
            if miss:
                bad += 1
                print("seed %d %s: %d mismatches %s" % (sd, name, len(miss), miss[:3]), flush=True)
        if sd % 10 == 9:
            print("%d seeds, %d requests, %d calls with mismatches, %.1f s" % (sd - 999, total, bad,
                  time.perf_counter() - t0), flush=True)
    print("calls with mismatches", bad, flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
