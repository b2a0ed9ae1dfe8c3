"""Diagnostic (round 5): the C3-many-sets workload of tests/test_gpu_configs.py
(test_c3_many_sets_through_the_cache[40-2050-70000]) run several times in ONE process, on fresh
cache-on and cache-off contexts, counting outcome mismatches against the oracle loops per call.
One closing session saw a single false "wrong signature" in the first (generic) call; this
measures how often, and on which path.  Usage: python tools/stress/c3_flake.py [trials]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

os.environ["TMED_PIPE_SIGS"] = "70000"

from conftest import engine_with_env  # noqa: E402
from test_gpu_configs import CHAIN, T2023, _bid, _corrupt, _ocommit, _oracle, _ovals, _same  # noqa: E402
import tmed.types as T  # noqa: E402
from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits  # noqa: E402


def workload(eng, nv=40, H=2050, gap=2):
    seeds = seeds_from_tag(b"tmed-c3-many", 0, H + gap + nv)
    pubs = pubkeys_of(eng, seeds)
    sets, specs = {}, []
    for h in range(H + gap):
        vals, order = make_valset(pubs[h:h + nv], [10] * nv)
        sets[h] = vals
        addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
        specs.append((seeds[h:h + nv][order], addrs, h + 1, 0, _bid(b"c3m-%d" % (h + 1)), T2023 + h, None))
    commits = dict(zip(range(H + gap), sign_commits(eng, CHAIN, specs)))
    for h, i in ((7, 1), (1000, 5), (2049, 0), (1500, nv - 1)):
        _corrupt(commits[h], i)
    reqs, exp, osets = [], [], {h: _ovals(v) for h, v in sets.items()}
    for h in range(H):
        u = h + gap
        pc = commits[u]
        oc = _ocommit(pc)
        for req, ovs in (((T.MODE_LIGHT_TRUSTING, sets[h], CHAIN, None, 0, pc, 1, 3), osets[h]),
                         ((T.MODE_LIGHT, sets[u], CHAIN, pc.block_id, u + 1, pc, 0, 0), osets[u])):
            reqs.append(req)
            exp.append(_oracle(req, ovs, oc))
    return reqs, exp


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    base = engine_with_env()
    reqs, exp = workload(base)
    base.close()
    total = 0
    for t in range(trials):
        cache = t % 3 != 2  # two cache-on trials for every cache-off one
        e = engine_with_env(TMED_KEYCACHE=1 if cache else 0)
        if cache:
            e.keycache_config(True, 16 << 30)
        for call in range(3):
            t0 = time.perf_counter()
            got = T.verify_commits(e, reqs)
            if cache:
                e.keycache_wait()
            bad = [(q, str(got[q]), str(exp[q])) for q in range(len(reqs)) if not _same(got[q], exp[q])]
            total += len(bad)
            print("trial %d cache %d call %d: %d mismatches %.3f s %s" % (t, cache, call, len(bad),
                  time.perf_counter() - t0, bad[:3]), flush=True)
        e.close()
    print("total mismatches", total, flush=True)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
