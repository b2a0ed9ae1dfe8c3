"""N>1 path on CPU: two gloo ranks shard a batch of commits, verify their shards through the
C++ seam (oracle as the batch verifier — no GPU here), all-reduce the int64 tallies and
all-gather the decisions; the result must equal the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _requests():
    from commit_cases import pbid, scenarios
    reqs, exp = [], []
    from commit_cases import oracle_result
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=9, count=24):
        reqs.append((mode, pv, chain, pbid(bid), h, pc, num, den))
        exp.append(oracle_result(mode, vs, chain, bid, h, cm, num, den))
    return reqs, exp


def _verifier(pubs, sigs, lens, msgs, offs):
    from oracle import port
    out = port.verify_batch(pubs, sigs, msgs, offs.astype(np.uint64), 2)
    out[lens != 64] = 0
    return out


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tendermint-fork_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from tmed.dist import verify_sharded
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    reqs, exp = _requests()
    r = verify_sharded(None, reqs, rank, world, verifier=_verifier)
    q.put((rank, r["ok"], r["commits"], r["verified"], r["codes"].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_tallies_match_single_process(world):
    import torch.distributed as dist  # noqa: F401
    from tmed.dist import shard
    reqs, exp = _requests()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp_ok = sum(e is None for e in exp)
    exp_codes = [0 if e is None else 1 for e in exp]
    for rank, ok, n, verified, codes in res:
        assert ok == exp_ok and n == len(reqs)
        assert codes == exp_codes
    assert sorted(sum((shard(len(reqs), r, world) for r in range(world)), [])) == list(range(len(reqs)))


def _sliced_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tendermint-fork_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from commit_cases import pbid, scenarios
    from tmed.dist import verify_commit_sliced
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    out = []
    for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=17, count=30):
        err, m = verify_commit_sliced(None, (mode, pv, chain, pbid(bid), h, pc, num, den), rank, world,
                                      verifier=_verifier_slice)
        out.append((None if err is None else (type(err).__name__, str(err)), m))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _verifier_slice(pubs, sigs, lens, msgs, offs):
    return _verifier(pubs, sigs, lens, msgs, offs)


@pytest.mark.parametrize("world", [2, 3])
def test_index_sliced_commit_matches_reference_loop(world):
    """§8e latency mode: one commit's candidates split over the ranks, one all-reduce MIN of
    the first failing index; every rank must return the reference loop's exact error."""
    from commit_cases import oracle_result, scenarios
    exp = [oracle_result(mode, vs, chain, bid, h, cm, num, den)
           for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=17, count=30)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sliced_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    kinds = set()
    for rank, out in res:
        for (got, m), e in zip(out, exp):
            want = None if e is None else (type(e).__name__, str(e))
            assert got == want, (rank, got, want)
            kinds.add("ok" if e is None else type(e).__name__)
    assert len(kinds) >= 3, kinds  # ok, wrong-signature and not-enough-power cases all crossed slices


def _blocksync_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tendermint-fork_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from tmed.dist import aggregate_blocksync, block_range
    from tmed.types import verify_commits
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    reqs = _light_blocks()
    lo, hi = block_range(len(reqs), rank, world)
    stats = []
    errs = verify_commits(None, reqs[lo:hi], verifier=_verifier, stats=stats) if hi > lo else []
    ok_bits = np.array([e is None for e in errs], np.uint8)
    agg = aggregate_blocksync(ok_bits, len(reqs), rank, world, sum(stats), mismatches=rank,
                              seconds=1.0 + rank, extra_max=[0.25 * (rank + 1)], phases=[10.0 * rank, 1.0, 2.0],
                              per_rank=[rank % 2, 64, 8, 13 - rank, rank, 0.5 + rank, 1000.0 * (rank + 1), 0])
    q.put((rank, agg["blocks_ok"], agg["blocks"], agg["verified"], agg["mismatches"], agg["seconds"],
           agg["extra_max"], agg["ok_bits"].tolist(), agg["phases"], agg["per_rank"]))
    dist.barrier()
    dist.destroy_process_group()


def _light_blocks():
    """Blocksync-shaped requests (VerifyCommitLight per block) from the seeded commit scenarios."""
    import tmed.types as T
    from commit_cases import pbid, scenarios
    return [(T.MODE_LIGHT, pv, chain, pbid(bid), h, pc, num, den)
            for mode, vs, pv, chain, bid, h, cm, pc, num, den in scenarios(seed=23, count=60) if mode == T.MODE_LIGHT]


@pytest.mark.parametrize("world", [2, 8])  # 8: the driver's node (21 blocks: uneven shards of 2 and 3)
def test_blocksync_aggregation_matches_single_process(world):
    """bench.py's C4 collectives (tmed.dist.aggregate_blocksync): contiguous block ranges per rank,
    ONE int64 all-reduce of (blocks ok, blocks, verified, mismatches), a MAX of the seam (and
    marshal) times, ONE all-gather of the packed decision bitmaps — equal to one process verifying
    every block (stub verifier: the C port)."""
    from tmed.types import verify_commits
    reqs = _light_blocks()
    assert len(reqs) >= 5
    stats = []
    single = np.array([e is None for e in verify_commits(None, reqs, verifier=_verifier, stats=stats)], np.uint8)
    assert 0 < single.sum() < len(reqs)  # ok and failing blocks both present
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_blocksync_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, nb, ver, mism, sec, extra, bits, phases, per_rank in res:
        assert (ok, nb, ver) == (int(single.sum()), len(reqs), sum(stats))
        assert mism == sum(range(world)) and sec == 1.0 + (world - 1) and extra == [0.25 * world]
        assert bits == single.tolist()
        assert [p[0] for p in phases] == [10.0 * r for r in range(world)] and all(p[-1] == 1.0 + r for r, p in enumerate(phases))
        # every rank's placement, memory mode and overlapped-marshal pass reach every rank (C4's
        # per-rank report): the whole-job overlapped rate is all ranks' verifies / the slowest rank
        assert per_rank == [[r % 2, 64, 8, 13 - r, r, 0.5 + r, 1000.0 * (r + 1), 0] for r in range(world)]
        from tmed.dist import overlapped_figures
        value, each = overlapped_figures(per_rank, 5, 6)
        assert value == round(sum(1000.0 * (r + 1) for r in range(world)) / (0.5 + world - 1), 1)
        assert each == [round(1000.0 * (r + 1) / (0.5 + r), 1) for r in range(world)]


def test_rehearsal_lines_name_simulated_gpus(monkeypatch):
    """A gloo rehearsal with more ranks than GPUs labels its JSON n_gpus_simulated /
    n_gpus_physical (bench.py, bench_commits.py); a real run keeps n_gpus."""
    import torch
    from tmed.launch import gpu_count_fields
    ndev = max(1, torch.cuda.device_count())
    monkeypatch.setenv("TMED_DIST_BACKEND", "gloo")
    assert gpu_count_fields(ndev + 1) == {"n_gpus_simulated": ndev + 1, "n_gpus_physical": ndev}
    assert gpu_count_fields(1) == {"n_gpus": 1}
    monkeypatch.delenv("TMED_DIST_BACKEND")
    assert gpu_count_fields(ndev + 1) == {"n_gpus": ndev + 1}
