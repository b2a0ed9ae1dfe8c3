"""Diagnostic (round 5): the blocksync window stream (tmed_blocksync_submit / _wait) many times on
one context, key-cached (batches alternating the two kernel lanes) and generic, every window's
codes and verified counts compared with a per-window run on a second, generic context.  The
workload is tests/test_gpu_commit.py's stream test (1,500 validators, windows of 12, 1, 5, 12 and
7 blocks, pinned and pageable signatures, bad signatures before and after the crossing).
Usage: python tools/stress/bs_stress.py [iterations]"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from conftest import engine_with_env  # noqa: E402
import tmed.types as T  # noqa: E402
from tmed import PinnedBuffer  # noqa: E402
from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    eng, ref_eng = engine_with_env(), engine_with_env()
    nvals = 1500
    seeds = seeds_from_tag(b"tmed-stream-key", 0, nvals)
    vals, order = make_valset(pubkeys_of(eng, seeds), [10] * nvals)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    upto = nvals * 2 // 3 + 1
    bufs, wins, b0 = [], [], 0
    for k, n in enumerate([12, 1, 5, 12, 7]):
        bids = [T.BlockID(hashlib.sha256(b"st%d" % b).digest(), 3, hashlib.sha256(b"sp%d" % b).digest())
                for b in range(b0, b0 + n)]
        specs = [(seeds[order], addrs, 500 + b, 0, bids[b - b0], 1672531200 + b, None) for b in range(b0, b0 + n)]
        commits = sign_commits(eng, "stream-chain", specs, sign_upto=upto)
        for b, c in zip(range(b0, b0 + n), commits):
            if b % 4 == 1:
                c.sigs[(b * 37) % upto, 5] ^= 0x20
            if b % 6 == 2:
                c.sigs[upto + 3, 1] ^= 0x02
        if k % 2 == 0:
            buf = PinnedBuffer(n * nvals * 64)
            a = buf.array((n * nvals, 64), np.uint8)
            for j, c in enumerate(commits):
                a[j * nvals:(j + 1) * nvals] = c.sigs
                c.sigs = a[j * nvals:(j + 1) * nvals]
            bufs.append(buf)
        wins.append((bids, [500 + b for b in range(b0, b0 + n)], commits))
        b0 += n
    ref = []
    for bids, hs, commits in wins:
        w = T.BlocksyncWindow(vals, "stream-chain", bids, hs, commits)
        w.run(ref_eng, 2)
        ref.append((w.codes().copy(), w.verified().copy()))
    ks = eng.keyset_load(np.array([np.frombuffer(v.pub_key, np.uint8) for v in vals.validators]))
    kvals = T.ValidatorSet(list(vals.validators))
    kvals.keyset = ks
    bad, t0 = 0, time.perf_counter()
    for it in range(iters):
        for vs, bb in ((kvals, 2), (kvals, 8), (vals, 2), (vals, 8)):  # 8 blocks: throughput kernels, two lanes
            ws = [T.BlocksyncWindow(vs, "stream-chain", bids, hs, commits) for bids, hs, commits in wins]
            for w in ws:
                w.submit(eng, bb)
            T.blocksync_wait(eng)
            for k, w in enumerate(ws):
                if not ((w.codes() == ref[k][0]).all() and (w.verified() == ref[k][1]).all()):
                    bad += 1
                    print("iteration %d keyed %d batch %d window %d differs: %s / %s" % (it, vs is kvals, bb, k, w.codes(), ref[k][0]),
                          flush=True)
        if it % 50 == 49:
            print("%d iterations, %d window mismatches, %.1f s" % (it + 1, bad, time.perf_counter() - t0), flush=True)
    eng.keyset_free(ks)
    print("total window mismatches", bad, flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
