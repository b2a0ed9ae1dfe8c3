"""Diagnostic (round 5): the opt-in ZIP-215 batch mode (randomized batch equations with a fresh
CSPRNG draw per call, bisection, single checks) on a 200k-signature batch with 0-6 fresh bit flips
per call, repeated, every decision compared with the C port's ZIP-215 rule (the base batch checked
once in full, the flipped signatures each call); "go" runs the default rule through the generic
kernels the same way, "keyed" through the key-cached kernels (1,000 keys), "small" with calls of
1..4,096 signatures (the latency kernels), generic and keyed alternately.
Usage: python tools/stress/zip_stress.py [calls] [go|keyed|small]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from conftest import engine_with_env  # noqa: E402
from oracle import port  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    small = "small" in sys.argv[2:]  # calls of 1..4,096 signatures (latency kernels), generic and keyed alternately
    keyed = "keyed" in sys.argv[2:] or small  # the default rule through the key-cached kernels (1,000 keys)
    z = "go" not in sys.argv[2:] and not keyed  # "go": the default (Go 1.18) rule, generic kernels
    e = engine_with_env()
    n = 200_000
    rng = np.random.default_rng(215)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    vi = rng.integers(0, 1000, n).astype(np.uint32)
    if keyed:
        seeds = seeds[:1000][vi]
    offs = (np.arange(n + 1) * 114).astype(np.uint32)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = e.sign_arrays(seeds, msgs, offs)
    ks = 0
    if keyed:  # key j's encoding from its first signature (every key is used: 200k draws of 1,000)
        u, first = np.unique(vi, return_index=True)
        assert u.size == 1000
        ks = e.keyset_load(np.ascontiguousarray(pubs[first]))
    base = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16, zip215=z)
    bad, t0 = 0, time.perf_counter()
    for c in range(calls):
        k = int(rng.integers(0, 7))
        m = int(rng.integers(1, 4097)) if small else n
        lo = int(rng.integers(0, n - m)) if small else 0
        idx = lo + np.unique(rng.integers(0, m, k))
        saved = sigs[idx].copy()
        for i in idx:
            sigs[i, int(rng.integers(0, 64))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        exp = base.copy()
        if idx.size:
            sub_off = np.zeros(idx.size + 1, np.uint64)
            sub_off[1:] = 114 * np.arange(1, idx.size + 1)
            sub_msgs = np.concatenate([msgs[offs[i]:offs[i] + 114] for i in idx] + [np.zeros(16, np.uint8)])
            exp[idx] = port.verify_batch(pubs[idx], sigs[idx], sub_msgs, sub_off, 1, zip215=z)
        if small:
            so = (offs[lo:lo + m + 1] - offs[lo]).astype(np.uint32)
            sm = np.ascontiguousarray(msgs[offs[lo]:offs[lo + m] + 16])
            out = (e.verify_keyset_arrays(ks, vi[lo:lo + m], sigs[lo:lo + m], sm, so) if c % 2 else
                   e.verify_arrays(pubs[lo:lo + m], sigs[lo:lo + m], sm, so))
            exp = exp[lo:lo + m]
        elif keyed:
            out = e.verify_keyset_arrays(ks, vi, sigs, msgs, offs)
        else:
            out = e.verify_zip215_arrays(pubs, sigs, msgs, offs) if z else e.verify_arrays(pubs, sigs, msgs, offs)
        diff = np.nonzero(out != exp)[0]
        if diff.size:
            bad += 1
            print("call %d: %d mismatches at %s (flipped %s)" % (c, diff.size, diff[:8], idx), flush=True)
        sigs[idx] = saved
        if c % 25 == 24:
            print("%d calls, %d with mismatches, %.1f s" % (c + 1, bad, time.perf_counter() - t0), flush=True)
    e.close()
    print("calls with mismatches", bad, flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
