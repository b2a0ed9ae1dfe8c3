"""Host placement of one rank per GPU on a multi-socket node (bench.py / bench_commits.py C4;
SURVEY.md §8e): each rank's seam threads, pinned staging arenas and Python harness belong on the
NUMA node its GPU hangs off, so an 8-rank node runs the same host path as a 1-rank box.

The GPU a rank drives is found WITHOUT touching the GPU (a HIP call would start the runtime's
threads with the old CPU mask, and nothing may exec after it): the KFD topology lists the GPU
agents in the order HIP enumerates them (nodes with a non-zero gpu_id, by node number), narrowed
by ROCR_VISIBLE_DEVICES then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (index lists); the
agent's PCI location (domain, location_id = bus << 8 | device << 3 | function) names its
/sys/bus/pci/devices entry, whose numa_node names /sys/devices/system/node/node<k>/cpulist.

bind_rank() then restricts the calling process (before any thread of the HIP runtime or of the
seam's host pool exists, so they all inherit it) to that node's CPUs that the process may use,
and sizes the seam's host pool (TMED_HOST_THREADS) to those CPUs shared among the node's ranks.
Pure sysfs reads: everything returns None (and binds nothing) where a file is missing."""
from __future__ import annotations

import os


def _read(path: str):
    try:
        with open(path) as fh:
            return fh.read()
    except OSError:
        return None


def parse_cpulist(s: str) -> list:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (the kernel's cpulist format)."""
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _visible(env: dict, n: int) -> list | None:
    """Device indexes after the visibility variables (None: a form other than an index list)."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None or v.strip() == "":
            continue
        try:
            sel = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:  # UUIDs: not resolved here
            return None
        if any(k < 0 or k >= len(idx) for k in sel):
            return None
        idx = [idx[k] for k in sel]
        if var == "ROCR_VISIBLE_DEVICES":
            continue
        break  # HIP_VISIBLE_DEVICES wins over CUDA_VISIBLE_DEVICES
    return idx


def gpu_agents(sysfs: str = "/sys") -> list:
    """[(kfd node, pci bdf 'dddd:bb:dd.f')] of the GPU agents in HIP's enumeration order."""
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        nodes = sorted((int(d) for d in os.listdir(base) if d.isdigit()))
    except OSError:
        return []
    out = []
    for k in nodes:
        gid = _read(os.path.join(base, str(k), "gpu_id"))
        if gid is None or int(gid.strip() or 0) == 0:
            continue
        props = {}
        for line in (_read(os.path.join(base, str(k), "properties")) or "").splitlines():
            f = line.split()
            if len(f) == 2:
                props[f[0]] = int(f[1])
        if "location_id" not in props:
            continue
        loc, dom = props["location_id"], props.get("domain", 0)
        out.append((k, "%04x:%02x:%02x.%d" % (dom, (loc >> 8) & 0xFF, (loc >> 3) & 0x1F, loc & 0x7)))
    return out


def gpu_numa_node(local_rank: int, sysfs: str = "/sys", env: dict | None = None):
    """(pci bdf, numa node) of the GPU that local_rank drives, or None."""
    env = os.environ if env is None else env
    agents = gpu_agents(sysfs)
    vis = _visible(env, len(agents))
    if not agents or vis is None or local_rank >= len(vis):
        return None
    bdf = agents[vis[local_rank]][1]
    s = _read(os.path.join(sysfs, "bus", "pci", "devices", bdf, "numa_node"))
    if s is None:
        return None
    node = int(s.strip())
    return (bdf, node) if node >= 0 else None


def visible_gpu_count(sysfs: str = "/sys", env: dict | None = None):
    """GPUs this process will see (KFD agents narrowed by the visibility variables), read without
    touching the HIP runtime; None when the topology or the variables cannot be resolved."""
    env = os.environ if env is None else env
    agents = gpu_agents(sysfs)
    vis = _visible(env, len(agents))
    if not agents or vis is None:
        return None
    return len(vis)


def node_cpus(node: int, sysfs: str = "/sys") -> list:
    s = _read(os.path.join(sysfs, "devices", "system", "node", "node%d" % node, "cpulist"))
    return parse_cpulist(s) if s else []


def plan_binding(local_rank: int, local_world: int, sysfs: str = "/sys", env: dict | None = None,
                 allowed: set | None = None, ndev: int | None = None) -> dict | None:
    """Where local_rank should run: {"gpu_bdf", "numa_node", "cpus" (sorted list), "host_threads",
    "ranks_on_node"}, or None when the topology cannot be read.  cpus = the node's CPUs that the
    process may use (`allowed`, default its current affinity); host_threads = those CPUs divided
    among the local ranks whose GPUs share the node (at least 2, at most 16: one GPU's share).
    ndev: local rank r drives device r % ndev (a gloo rehearsal of more ranks than GPUs)."""
    me = gpu_numa_node(local_rank, sysfs, env)
    if me is None:
        return None
    bdf, node = me
    allowed = set(os.sched_getaffinity(0)) if allowed is None else set(allowed)
    cpus = sorted(set(node_cpus(node, sysfs)) & allowed)
    if not cpus:
        return None
    peers = 0
    for r in range(max(1, local_world)):
        g = gpu_numa_node(r % ndev if ndev else r, sysfs, env)
        if g is not None and g[1] == node:
            peers += 1
    peers = max(1, peers)
    threads = max(2, min(16, len(cpus) // peers))
    return {"gpu_bdf": bdf, "numa_node": node, "cpus": cpus, "host_threads": threads, "ranks_on_node": peers}


def bind_rank(local_rank: int, local_world: int, ndev: int | None = None) -> dict:
    """Bind this process to its GPU's NUMA node (os.sched_setaffinity, no exec) and set
    TMED_HOST_THREADS unless the caller set it.  Call before anything touches the GPU.
    TMED_BIND=0 turns it off.  Returns what was done (reported per rank by the benches)."""
    if os.environ.get("TMED_BIND", "1") == "0":
        return {"bound": False, "reason": "TMED_BIND=0"}
    plan = plan_binding(local_rank, local_world, ndev=ndev)
    if plan is None:
        return {"bound": False, "reason": "GPU topology not readable (no KFD / PCI numa_node)",
                "cpus_allowed": len(os.sched_getaffinity(0))}
    try:
        os.sched_setaffinity(0, plan["cpus"])
    except OSError as e:
        return {"bound": False, "reason": "sched_setaffinity: %s" % e, **_brief(plan)}
    if "TMED_HOST_THREADS" not in os.environ:
        os.environ["TMED_HOST_THREADS"] = str(plan["host_threads"])
    return {"bound": True, **_brief(plan), "host_threads_env": os.environ["TMED_HOST_THREADS"]}


def cgroup_cpu_stat(path: str = "/sys/fs/cgroup/cpu.stat") -> dict | None:
    """The cgroup v2 CPU counters of this process's group ({"usage_usec", "nr_periods",
    "nr_throttled", "throttled_usec", ...} as ints), or None where the file is missing.  A GPU box
    grants a job CPU bandwidth (cpu.max), not a CPU set: threads may run on any CPU, and once the
    group has used its quota in a period ALL its threads stop until the next one."""
    s = _read(path)
    if s is None:
        return None
    out = {}
    for line in s.splitlines():
        k, _, v = line.partition(" ")
        try:
            out[k] = int(v)
        except ValueError:
            pass
    return out


def cgroup_delta(before: dict | None, after: dict | None, wall_s: float) -> dict | None:
    """What a timed region cost the group: CPUs in use on average, throttled periods and the time
    the group stood throttled (None without cgroup counters)."""
    if not before or not after:
        return None
    d = {k: after.get(k, 0) - before.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec")}
    return {"cpus_used": round(d["usage_usec"] / 1e6 / wall_s, 2) if wall_s > 0 else None,
            "periods": d["nr_periods"], "throttled_periods": d["nr_throttled"],
            "throttled_ms": round(d["throttled_usec"] / 1e3, 3)}


def _brief(plan: dict) -> dict:
    c = plan["cpus"]
    return {"gpu_bdf": plan["gpu_bdf"], "numa_node": plan["numa_node"], "cpus": len(c),
            "cpu_range": "%d-%d" % (c[0], c[-1]), "host_threads": plan["host_threads"],
            "ranks_on_node": plan["ranks_on_node"]}
