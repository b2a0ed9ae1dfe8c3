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


def _collectives(world: int) -> bool:
    """Whether the ranks exchange: always at world > 1, and at world 1 when a process group exists
    (a one-rank RCCL group runs the same collectives, dtypes and devices as an N-rank one:
    tests/test_gpu_rccl.py)."""
    if world > 1:
        return True
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


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
    if _collectives(world):
        dist.all_reduce(tally)
        gathered = [torch.empty_like(full) for _ in range(world)]
        dist.all_gather(gathered, full)
        full = torch.stack(gathered).max(dim=0).values  # each slot owned by exactly one rank
    ok, n, verified = (int(x) for x in tally.tolist())
    return {"ok": ok, "commits": n, "verified": verified, "codes": full.cpu().numpy()}


def slice_bounds(m: int, rank: int, world: int) -> tuple:
    """Contiguous candidate slice [lo, hi) of `rank` (sizes differ by at most one)."""
    return m * rank // world, m * (rank + 1) // world


def verify_commit_sliced(engine, request: tuple, rank: int, world: int, device=None, verifier=None):
    """Latency mode for ONE large commit: the validator index range is split
    over the ranks instead of whole commits.

    Every rank runs the seam on the whole commit — prechecks, candidate selection and
    sign-bytes are host work and identical everywhere — but verifies only its contiguous
    slice of the candidates.  The ranks then agree on f, the first failing candidate, with
    ONE int64 all-reduce MIN, and every rank replays the reference loop with bits "valid
    before f, invalid at f".  The loop never looks past f: VerifyCommit errors at f
    (types/validator_set.go:695-698), and Light/Trusting either crossed 2/3 before f or error
    at f (:751-761, :812-822), so the error, its index and Got/Needed equal the
    single-process result.  (The power tally needs no collective: every rank holds the
    commit.)  Returns the Go-style error (None = ok) and the number of candidates."""
    import torch
    import torch.distributed as dist
    from .types import verify_commits

    dev = device if device is not None else torch.device("cpu")
    seen = []

    def sliced(pubs, sigs, lens, msgs, offs):
        m = pubs.shape[0]
        lo, hi = slice_bounds(m, rank, world)
        first = m
        if hi > lo:
            o = offs[lo:hi + 1].astype(np.int64)
            sub_msgs = msgs[o[0]:o[-1]]
            sub_offs = (o - o[0]).astype(np.uint32)
            if verifier is None:
                bits = engine.verify_arrays(pubs[lo:hi], sigs[lo:hi], sub_msgs, sub_offs, lens[lo:hi])
            else:
                bits = np.asarray(verifier(pubs[lo:hi], sigs[lo:hi], lens[lo:hi], sub_msgs, sub_offs), np.uint8)
            bad = np.flatnonzero(bits == 0)
            if bad.size:
                first = lo + int(bad[0])
        f = torch.tensor([first], dtype=torch.int64, device=dev)
        if _collectives(world):
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
        f = int(f.item())
        out = np.ones(m, np.uint8)
        if f < m:
            out[f] = 0
        seen.append(m)
        return out

    err = verify_commits(engine, [request], verifier=sliced)[0]
    return err, (seen[0] if seen else 0)


def block_range(blocks: int, rank: int, world: int) -> tuple:
    """Contiguous block heights [lo, hi) of `rank` for a blocksync replay (C4: 100k blocks / 8 GPUs)."""
    return blocks * rank // world, blocks * (rank + 1) // world


def aggregate_blocksync(ok_bits: np.ndarray, blocks: int, rank: int, world: int, verified: int, mismatches: int,
                        seconds: float, extra_max=(), phases=(), device=None, per_rank=()) -> dict:
    """The only collectives of a sharded blocksync replay: ONE int64 all-reduce of
    the tallies (blocks ok, blocks, signatures verified, outcome mismatches), a MAX of the ranks' seam
    times (and of `extra_max`, e.g. marshalling times), ONE all-gather of the per-block decision
    bitmaps (packed bits, every rank padded to the largest shard) and of the per-rank `phases`
    (diagnostics) and of `per_rank` (this rank's placement and memory mode: NUMA node, CPUs, host
    threads, pinned / pageable arenas — so an N-rank line cannot hide one rank on another path).
    ok_bits: this rank's blocks [lo, hi) of block_range.  Returns the same dict on every rank;
    "ok_bits" is the whole chain's bitmap in height order, "per_rank" one list per rank."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else torch.device("cpu")
    lo, hi = block_range(blocks, rank, world)
    assert ok_bits.shape[0] == hi - lo
    tally = torch.tensor([int(ok_bits.sum()), hi - lo, int(verified), int(mismatches)], dtype=torch.int64, device=dev)
    tmax = torch.tensor([float(seconds)] + [float(x) for x in extra_max], dtype=torch.float64, device=dev)
    per = -(-blocks // world)  # the largest shard
    bits = torch.from_numpy(np.packbits(np.pad(ok_bits.astype(np.uint8), (0, per - (hi - lo))))).to(dev)
    ph = torch.tensor([float(x) for x in phases] + [float(seconds)], dtype=torch.float64, device=dev)
    pr = torch.tensor([float(x) for x in per_rank] + [float(rank)], dtype=torch.float64, device=dev)
    if _collectives(world):
        dist.all_reduce(tally)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        gb = [torch.empty_like(bits) for _ in range(world)]
        dist.all_gather(gb, bits)
        gp = [torch.empty_like(ph) for _ in range(world)]
        dist.all_gather(gp, ph)
        gr = [torch.empty_like(pr) for _ in range(world)]
        dist.all_gather(gr, pr)
    else:
        gb, gp, gr = [bits], [ph], [pr]
    full = []
    for r in range(world):
        a, b = block_range(blocks, r, world)
        full.append(np.unpackbits(gb[r].cpu().numpy())[:b - a])
    ok, nb, ver, mism = (int(x) for x in tally.tolist())
    tm = tmax.tolist()
    return {"blocks_ok": ok, "blocks": nb, "verified": ver, "mismatches": mism, "seconds": tm[0],
            "extra_max": tm[1:], "ok_bits": np.concatenate(full) if full else np.zeros(0, np.uint8),
            "phases": [g.tolist() for g in gp], "per_rank": [g.tolist()[:-1] for g in gr]}


def overlapped_figures(per_rank, seconds_idx: int, verifies_idx: int):
    """The drop-in's host cost at N ranks (bench_commits.c4, the overlapped-marshal pass every rank
    runs): (whole-job verifies/s = every rank's verifies / the slowest rank's seconds, [each rank's own
    verifies/s]) from aggregate_blocksync's per_rank rows.  None values where a rank ran no pass."""
    secs = [float(p[seconds_idx]) for p in per_rank]
    vers = [float(p[verifies_idx]) for p in per_rank]
    each = [round(v / t, 1) if t > 0 else None for v, t in zip(vers, secs)]
    tmax = max(secs) if secs else 0.0
    return (round(sum(vers) / tmax, 1) if tmax > 0 else None), each
