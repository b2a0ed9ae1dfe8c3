#!/usr/bin/env python3
"""Crossover of the key-cached latency kernels vs the throughput kernels: p50 wall time of
tmed_verify_batch_keyset_device (inputs resident in HBM, synchronised per call) at several
batch sizes, one engine per path (TMED_LAT_MAX=65536 vs 0).  Prints one JSON line per size."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))


def engine(lat_max):
    from tmed import Engine
    os.environ["TMED_LAT_MAX"] = str(lat_max)
    e = Engine(0)
    del os.environ["TMED_LAT_MAX"]
    return e


def main():
    import torch
    from tmed.workload import c2_messages, seeds_from_tag
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "175,1024,4096,16384,65536").split(",")]
    dev = torch.device("cuda", 0)
    nmax, nk = max(sizes), 1000
    kseeds = seeds_from_tag(b"tmed-lat-key", 0, nk)
    val_idx = (np.arange(nmax) % nk).astype(np.uint32)
    msgs, offs = c2_messages(0, nmax)
    engs = {"latency": engine(65536), "throughput": engine(0)}
    e0 = engs["latency"]
    d_seed = torch.from_numpy(kseeds[val_idx]).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_sig = torch.empty((nmax, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((nmax, 32), dtype=torch.uint8, device=dev)
    d_vi = torch.from_numpy(val_idx.view(np.int32)).to(dev)
    e0.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, nmax, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    pubs = d_pub[:nk].cpu().numpy()
    hs = {k: e.keyset_load(pubs) for k, e in engs.items()}
    for n in sizes:
        row = {"n": n}
        outs = {}
        for k, e in engs.items():
            d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
            reps = 200 if n <= 4096 else 50
            ts = []
            for r in range(reps + 5):
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                e.verify_keyset_device(hs[k], d_vi, d_sig, d_msg, d_off, d_out, n)
                torch.cuda.synchronize(dev)
                if r >= 5:
                    ts.append(time.perf_counter() - t)
            row[k + "_p50_us"] = round(1e6 * float(np.median(ts)), 1)
            outs[k] = d_out.cpu().numpy()
        row["agree"] = bool((outs["latency"] == outs["throughput"]).all() and outs["latency"].all())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
