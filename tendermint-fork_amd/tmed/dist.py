"""Multi-GPU sharding of commit verification.

One process per GPU.  Independent commits (blocksync blocks, light-client headers) are
sharded round-robin over the ranks; each rank verifies its shard through the seam with
no data-path collective, then the per-rank int64 tallies (commits ok, commits, signatures
verified) are summed with ONE all-reduce (RCCL over xGMI on GPUs, gloo in the CPU tests),
and the per-commit decision bitmap is assembled with one all-gather.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def shard(n: int, rank: int, world: int) -> list:
    """Commit indices owned by `rank` (round-robin keeps every rank's load equal for uniform commits)."""
    return list(range(rank, n, world))


def verify_sharded(engine, requests: Sequence[tuple], rank: int, world: int, device=None, verifier=None):
    """Verify this rank's shard of `requests` (each a verify_commits tuple); return the global
    tallies and the global per-request outcome codes (identical on every rank)."""
    import torch
    import torch.distributed as dist
    from .types import PreparedBatch, verify_commits

    mine = shard(len(requests), rank, world)
    local = [requests[i] for i in mine]
    if verifier is None:
        pb = PreparedBatch(local)
        if local:
            pb.run(engine)
        codes = pb.codes() if local else np.zeros(0, np.int32)
        ver = pb.verified() if local else np.zeros(0, np.int64)
    else:
        stats = []
        errs = verify_commits(engine, local, verifier=verifier, stats=stats) if local else []
        codes = np.array([0 if e is None else 1 for e in errs], np.int32)
        ver = np.array(stats, np.int64)
    dev = device if device is not None else torch.device("cpu")
    tally = torch.tensor([int((codes == 0).sum()), len(local), int(ver.sum())], dtype=torch.int64, device=dev)
    full = torch.full((len(requests),), -1, dtype=torch.int32, device=dev)
    if mine:
        full[torch.tensor(mine, device=dev)] = torch.from_numpy(codes.astype(np.int32)).to(dev)
    if world > 1:
        dist.all_reduce(tally)
        gathered = [torch.empty_like(full) for _ in range(world)]
        dist.all_gather(gathered, full)
        full = torch.stack(gathered).max(dim=0).values  # each slot owned by exactly one rank
    ok, n, verified = (int(x) for x in tally.tolist())
    return {"ok": ok, "commits": n, "verified": verified, "codes": full.cpu().numpy()}
