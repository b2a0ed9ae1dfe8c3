"""Process-group setup shared by the benches: one process per GPU (torchrun env), RCCL over
xGMI for the small tally collectives.  TMED_DIST_BACKEND=gloo rehearses N ranks on fewer
GPUs (rank r uses device LOCAL_RANK % device_count, collectives run on CPU tensors) — how
the multi-rank paths are exercised on a one-GPU box; the driver's 8-GPU runs use RCCL."""
from __future__ import annotations

import os


BINDING: dict = {}  # this rank's host placement (tmed.affinity.bind_rank), reported by the benches


def dist_setup():
    """Returns (world, rank, local_rank, device, collective_device).  Before anything touches the
    GPU, the process is bound to the CPUs of its GPU's NUMA node (tmed.affinity.bind_rank; the
    result is kept in BINDING)."""
    import torch
    import torch.distributed as dist
    from .affinity import bind_rank
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    backend = os.environ.get("TMED_DIST_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())  # counts devices without initialising HIP (this image)
    local = local % ndev if backend == "gloo" else local
    BINDING.clear()
    BINDING.update(bind_rank(local, local_world, ndev))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll = dev
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            dist.init_process_group("gloo")
            coll = torch.device("cpu")
        else:
            dist.init_process_group("nccl", device_id=dev)
    return world, rank, local, dev, coll


def gpu_count_fields(world):
    """The JSON fields naming the GPU count of a run: {"n_gpus": world} for real ranks (one GPU
    each); for a gloo rehearsal with fewer GPUs than ranks, {"n_gpus_simulated": world,
    "n_gpus_physical": k} instead, so the line cannot be read as an N-GPU measurement."""
    import torch
    ndev = max(1, torch.cuda.device_count())
    if os.environ.get("TMED_DIST_BACKEND") == "gloo" and world > ndev:
        return {"n_gpus_simulated": world, "n_gpus_physical": ndev}
    return {"n_gpus": world}
