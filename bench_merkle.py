#!/usr/bin/env python3
"""bench_merkle.py — f3: batched SHA-256 Merkle roots on one MI355X, the
hashing either side of signature verification in the light client and blocksync:

  valset   ValidatorSet.Hash for 10,000 sets x 175 validators (light/verifier.go:183 hashes the
           untrusted set of every header: the C3 shape)
  headers  Header.Hash for 100,000 headers (light/verifier.go:237, blockchain/v0/reactor.go:359)
  partset  PartSet roots of 256 blocks x 1 MiB in 64 KiB parts (reactor.go:359-361 MakePartSet)

Each line: objects/s and hashed bytes/s end to end through the C ABI (host buffers in, roots
out: staging + H2D + kernels + D2H), next to the same work on one host core with hashlib
(OpenSSL SHA-256) through oracle/merkle.py on a bounded sample ("port", cpu_baseline only)."""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t)
    return min(ts), out


def cpu_rate(fn, items, budget_s=3.0):
    """Objects/s of fn over a growing prefix of items, about budget_s of one core."""
    n, dt = 1, 0.0
    while dt < budget_s / 4 and n <= len(items):
        t = time.perf_counter()
        for x in items[:n]:
            fn(x)
        dt = time.perf_counter() - t
        n *= 2
    return (n // 2) / dt, n // 2


def main():
    sys.path.insert(0, ROOT)
    from oracle import merkle as M  # cpu_baseline leg only
    from tmed import Engine
    from tmed import merkle as TM
    eng = Engine(0)
    rng = np.random.default_rng(1)
    res = []

    # valset: 10k x 175
    S, V = 10_000, 175
    pubs = rng.integers(0, 256, (S * V, 32), dtype=np.uint8)
    pows = np.full(S * V, 10, np.int64)
    off = (np.arange(S + 1) * V).astype(np.uint32)
    dt, got = timed(lambda: TM.valset_hashes_arrays(eng, pubs, pows, off))
    sets = [[(bytes(pubs[i]), 10) for i in range(s * V, (s + 1) * V)] for s in range(64)]
    assert all(bytes(got[s]) == M.valset_hash(sets[s]) for s in range(8))
    cpu, m = cpu_rate(M.valset_hash, sets)
    leaf_b = S * V * 39
    res.append({"metric": "ValidatorSet.Hash sets/s (175 validators)", "value": round(S / dt, 1), "unit": "sets/s",
                "leaf_bytes_per_s": round(leaf_b / dt, 1), "seconds": round(dt, 4),
                "cpu_baseline": {"value": round(cpu, 1), "unit": "sets/s", "cores": 1, "kind": "port",
                                 "sample": "%d sets, hashlib SHA-256 via oracle/merkle.py" % m},
                "config": {"workload": "f3 valset: %d sets x %d validators" % (S, V)}})

    # headers: 100k
    H = 100_000
    base = {"version_block": 11, "version_app": 1, "chain_id": "test_chain_id", "height": 1,
            "time": (1700000000, 5), "last_block_id": (bytes(32), 1, bytes(32))}
    hs = []
    for i in range(H):
        h = dict(base)
        h["height"] = i + 1
        h["time"] = (1700000000 + i, i % 1000)
        for k in M.HEADER_HASH_FIELDS:
            h[k] = hashlib.sha256(b"%s/%d" % (k.encode(), i)).digest()[: 20 if k == "proposer_address" else 32]
        hs.append(h)
    hb = TM.HeaderBatch(hs)                     # packed once: the timed region is the C call
    dt, got = timed(lambda: hb.run(eng), reps=2)
    assert all(got[i] == M.header_hash(hs[i]) for i in range(0, H, 9973))
    cpu, m = cpu_rate(M.header_hash, hs)
    res.append({"metric": "Header.Hash headers/s", "value": round(H / dt, 1), "unit": "headers/s",
                "seconds": round(dt, 4), "note": "C call: host-side field encoding (C++) + H2D + kernels + D2H",
                "cpu_baseline": {"value": round(cpu, 1), "unit": "headers/s", "cores": 1, "kind": "port",
                                 "sample": "%d headers" % m},
                "config": {"workload": "f3 headers: %d headers" % H}})

    # partset: 256 x 1 MiB
    B, SZ = 256, 1 << 20
    blocks = [rng.integers(0, 256, SZ, dtype=np.uint8).tobytes() for _ in range(B)]
    data = np.frombuffer(b"".join(blocks) + bytes(8), np.uint8)
    off = (np.arange(B + 1) * SZ).astype(np.uint64)
    dt, got = timed(lambda: TM.partset_roots_packed(eng, data, off, 65536))
    assert all(bytes(got[b]) == M.partset_root(blocks[b], 65536) for b in range(4))
    cpu, m = cpu_rate(lambda b: M.partset_root(b, 65536), blocks)
    res.append({"metric": "PartSet root bytes/s", "value": round(B * SZ / dt, 1), "unit": "B/s",
                "blocks_per_s": round(B / dt, 1), "seconds": round(dt, 4),
                "note": "end to end incl. %d MiB H2D over PCIe" % (B * SZ >> 20),
                "cpu_baseline": {"value": round(cpu * SZ, 1), "unit": "B/s", "cores": 1, "kind": "port",
                                 "sample": "%d blocks" % m},
                "config": {"workload": "f3 partset: %d blocks x 1 MiB, 64 KiB parts" % B}})
    for r in res:
        print(json.dumps(r), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
