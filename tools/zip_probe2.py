#!/usr/bin/env python3
"""ZIP-215 batch equation on all-valid batches: pass rate by size and seed (diagnostics)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
from tmed import Engine  # noqa: E402


def main():
    eng = Engine(0)
    rng = np.random.default_rng(5)
    nmax = 131072
    seeds = rng.integers(0, 256, (nmax, 32), dtype=np.uint8)
    offs = (np.arange(nmax + 1) * 114).astype(np.uint32)
    msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
    sigs, pubs = eng.sign_arrays(seeds, msgs, offs)
    for n in (20000, 24000, 28000, 32000, 32768, 33000, 40000, 65535, 65536, 65537, 80000, 131072):
        res = []
        for sd in range(3):
            Engine.zip215_set_seed(bytes([sd + 1] * 32))
            out = eng.verify_zip215_arrays(pubs[:n], sigs[:n], msgs, offs[:n + 1])
            st = Engine.zip215_stats()
            res.append((int(out.sum()), st["equations"]))
        print(json.dumps({"n": n, "res": res}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
