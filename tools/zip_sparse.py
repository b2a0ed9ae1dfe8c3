"""ZIP-215 batch mode with SPARSE failures (tools/zip_sparse.py): the cost of the batch-equation
path (full-chunk MSM, bisection to 2^14 groups, single checks of the failing groups) against the
single-check path, on 2^20 signatures with 0, 1, 4 and 16 invalid ones.  Each case: a fresh
context (batch equation first), then further calls on the same one (after a chunk with failures
the seam decides the next one singly, zip215.hip kZipSinglyMin).  One JSON line per case."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))


def main():
    import torch
    from tmed import Engine
    from tmed.workload import c2_messages, seeds_from_tag
    n = 1 << 20
    dev = torch.device("cuda:0")
    msgs, offs = c2_messages(0, n)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_seed = torch.from_numpy(seeds_from_tag(b"tmed-zip-sparse", 0, n)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    signer = Engine(0)
    signer.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n)
    torch.cuda.synchronize(dev)
    signer.close()
    rng = np.random.default_rng(5)
    for bad in (0, 1, 4, 16):
        sig = d_sig.clone()
        idx = rng.choice(n, bad, replace=False) if bad else np.zeros(0, np.int64)
        for i in idx:
            sig[int(i), 40] ^= 0x10
        eng = Engine(0)
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        eng.verify_zip215_device(d_pub, sig, d_msg, d_off, out, n)  # warm-up on a throwaway context
        torch.cuda.synchronize(dev)
        eng.close()
        eng = Engine(0)
        calls = []
        for c in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            eng.verify_zip215_device(d_pub, sig, d_msg, d_off, out, n)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) * 1e3
            got = out.cpu().numpy()
            ok = int((got == 0).sum()) == bad and all(got[int(i)] == 0 for i in idx)
            calls.append({"ms": round(ms, 3), "decisions_ok": bool(ok), "engine": Engine.zip215_stats()})
        eng.close()
        print(json.dumps({"invalid": bad, "n": n, "calls": calls}), flush=True)


if __name__ == "__main__":
    main()
