#!/usr/bin/env python3
"""bench_keyset.py — C2's second variant: 1,048,576 signatures by 10,000
validators with the per-validator-set key cache on (tmed_verify_batch_keyset_device: A decoded
once per key, [k](-A) from the key's signed radix-256 comb, no doublings), the path the commit
seam takes for blocksync (C4) and the light client (C3).  Inputs resident in HBM, one step =
one verification pass; prints one JSON line like bench.py (rank 0; N ranks = N shards)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))

MUL, SQ = 100, 55
sys.path.insert(0, ROOT)
from bench import mads_keyset_main  # noqa: E402  (rows of the key-cached main kernel -> mads)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--keys", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sorted", action="store_true", help="signatures ordered by validator index (as in a commit)")
    args = ap.parse_args()
    import torch
    from tmed import Engine
    from tmed.workload import c2_messages, seeds_from_tag
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    eng = Engine(local)
    n, nk = args.n, args.keys
    t_gen = time.time()
    kseeds = seeds_from_tag(b"tmed-c2k-key", 0, nk)
    rng = np.random.default_rng(7 + rank)
    val_idx = rng.integers(0, nk, n).astype(np.uint32)
    if args.sorted:
        val_idx = np.arange(n, dtype=np.uint32) % nk
    msgs, offs = c2_messages(rank * n, n)
    d_seed = torch.from_numpy(kseeds[val_idx]).to(dev)
    d_msg = torch.from_numpy(np.concatenate([msgs, np.zeros(16, np.uint8)])).to(dev)
    d_off = torch.from_numpy(offs.view(np.int32)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    d_pub = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_vi = torch.from_numpy(val_idx.view(np.int32)).to(dev)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    eng.sign_device(d_seed, d_msg, d_off, d_sig, d_pub, n, st.cuda_stream)
    torch.cuda.synchronize(dev)
    pubs = np.zeros((nk, 32), np.uint8)
    pub_all = d_pub.cpu().numpy()
    pubs[val_idx] = pub_all
    t_ks = time.perf_counter()
    ks = eng.keyset_load(pubs)
    t_ks = time.perf_counter() - t_ks
    t_gen = time.time() - t_gen

    def step():
        eng.verify_keyset_device(ks, d_vi, d_sig, d_msg, d_off, d_out, n, st.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ok_first = int(d_out.sum().item())
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    valid = int(d_out.sum().item())
    eng.set_kernel_timing(True)
    step()
    torch.cuda.synchronize(dev)
    (prep_ms, main_ms, fin_ms), (pl, ml, fl) = eng.kernel_times()
    eng.set_kernel_timing(False)
    kbits = eng.keyset_b_window_bits()
    abits = eng.keyset_a_window_bits(ks)
    eng.keyset_free(ks)
    eng.close()
    if rank == 0:
        print(json.dumps({
            "metric": "ed25519 verifies/sec at 1/8 MI355X (key-cached variant)", "value": round(n * args.steps / dt, 1),
            "unit": "verifies/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "all_valid": valid == n and ok_first == n, "keyset_build_s": round(t_ks, 3), "setup_s": round(t_gen, 2),
            "mads_per_verify_main": mads_keyset_main(kbits, abits), "b_window_bits": kbits, "a_window_bits": abits,
            "kernel_ms": {"prep": round(prep_ms, 4), "main": round(main_ms, 4), "finish": round(fin_ms, 4)},
            "sorted": args.sorted,
            "data": "synthetic (10k seeded keys, CanonicalVote sign-bytes, GPU RFC 8032 signer)",
            "config": {"workload": "C2 variant: %d signatures by %d validators, key cache on" % (n, nk)}}), flush=True)


if __name__ == "__main__":
    main()
