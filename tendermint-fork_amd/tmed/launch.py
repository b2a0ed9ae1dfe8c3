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
    from .affinity import bind_rank, visible_gpu_count
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    backend = os.environ.get("TMED_DIST_BACKEND", "nccl")
    # the device count comes from the KFD topology, so the binding happens before any torch.cuda
    # call: on a stock ROCm torch device_count() starts the HIP runtime's threads, which would keep
    # the old CPU mask (sched_setaffinity only rebinds the calling thread and its later children)
    ndev = visible_gpu_count()
    counted = "kfd"
    if ndev is None:
        ndev, counted = None, "unresolved"
    if ndev is not None:
        ndev = max(1, ndev)
        local = local % ndev if backend == "gloo" else local
    BINDING.clear()
    BINDING.update(bind_rank(local, local_world, ndev))
    if ndev is None:  # topology unreadable: nothing was bound, so counting through HIP is harmless now
        ndev = max(1, torch.cuda.device_count())
        local = local % ndev if backend == "gloo" else local
    BINDING["device_count_from"] = counted
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
