"""Latency probe (tools only): per-kernel device time of the generic verify path on small
batches (one lone wave per SIMD), to size the generic latency mode.  Prints one JSON line per n."""
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
    from tmed.workload import c2_messages, c2_seeds
    dev = torch.device("cuda:0")
    eng = Engine(0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    for n in [int(x) for x in (sys.argv[1:] or ["1", "64", "175", "1024"])]:
        seeds = c2_seeds(0, n)
        msgs, offs = c2_messages(0, n)
        d_seed = torch.from_numpy(seeds).to(dev)
        d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
        d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
        d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
        eng.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n, st.cuda_stream)
        torch.cuda.synchronize(dev)
        for _ in range(3):
            eng.verify_device(d_pub, d_sig, d_msg, d_off, d_out, n, st.cuda_stream)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            eng.verify_device(d_pub, d_sig, d_msg, d_off, d_out, n, st.cuda_stream)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        eng.set_kernel_timing(True)
        kt = []
        for _ in range(10):
            eng.verify_device(d_pub, d_sig, d_msg, d_off, d_out, n, st.cuda_stream)
            torch.cuda.synchronize(dev)
            kt.append(eng.kernel_times()[0])
        eng.set_kernel_timing(False)
        kt = np.median(np.array(kt), axis=0)
        print(json.dumps({"n": n, "all_ok": int(d_out.sum().item()) == n, "wall_p50_ms": round(float(np.median(ts)) * 1e3, 4),
                          "prep_ms": round(float(kt[0]), 4), "main_ms": round(float(kt[1]), 4),
                          "finish_ms": round(float(kt[2]), 4)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
