#!/usr/bin/env python3
"""Diagnostics of the opt-in ZIP-215 batch mode: for several batches, whether ONE batch equation
holds (tmed_zip215_stats) and whether the decisions equal the C port's ZIP-215 rule."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import port  # noqa: E402
from tmed import Engine  # noqa: E402
from test_gpu_zip215 import _pack, _zip_golden  # noqa: E402


def run(eng, name, pubs, sigs, msgs, offs):
    Engine.zip215_set_seed(bytes(range(32)))
    out = eng.verify_zip215_arrays(pubs, sigs, msgs, offs)
    st = Engine.zip215_stats()
    exp = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 16, zip215=True)
    print(json.dumps({"case": name, "n": int(pubs.shape[0]), "valid": int(exp.sum()),
                      "mismatch": int((out != exp).sum()), **st}), flush=True)


def main():
    eng = Engine(0)
    rng = np.random.default_rng(1)
    for n in (1, 2, 64, 1000, 20000, 100000):
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        offs = (np.arange(n + 1) * 114).astype(np.uint32)
        msgs = rng.integers(0, 256, int(offs[-1]) + 16, dtype=np.uint8)
        sigs, pubs = eng.sign_arrays(seeds, msgs, offs)
        run(eng, "valid", pubs, sigs, msgs, offs)
    gold = [it for it in _zip_golden() if it[4] == 1 and len(it[3]) == 64]
    classes = sorted({it[0] for it in gold})
    for c in classes:
        items = [it for it in gold if it[0] == c]
        p, s, _, m, o = _pack(items)
        run(eng, "class:" + c, p, s, m, o)
    eng.close()


if __name__ == "__main__":
    main()
