"""Host placement of one rank per GPU (tmed/affinity.py): KFD agent order -> PCI bus id -> NUMA
node -> the node's CPUs, on a synthetic sysfs tree shaped like a 2-socket, 8-GPU MI355X node
(GPUs 0-3 on node 0, 4-7 on node 1; node CPU lists with SMT siblings as lscpu shows them:
0-63,128-191 / 64-127,192-255).  CPU-only; no GPU is touched."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))

from tmed import affinity as A  # noqa: E402

BUSES = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5]  # one GPU per bus, in KFD node order


def _w(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write(text)


@pytest.fixture
def sysfs(tmp_path):
    root = str(tmp_path)
    kfd = os.path.join(root, "class", "kfd", "kfd", "topology", "nodes")
    # KFD nodes 0, 1: the CPU agents (gpu_id 0); nodes 2..9: the GPUs
    for k in range(2):
        _w(os.path.join(kfd, str(k), "gpu_id"), "0\n")
        _w(os.path.join(kfd, str(k), "properties"), "cpu_cores_count 128\nsimd_count 0\n")
    for g, bus in enumerate(BUSES):
        k = g + 2
        _w(os.path.join(kfd, str(k), "gpu_id"), "%d\n" % (1000 + g))
        _w(os.path.join(kfd, str(k), "properties"),
           "simd_count 1024\nlocation_id %d\ndomain 0\ndevice_id 30112\n" % (bus << 8))
        _w(os.path.join(root, "bus", "pci", "devices", "0000:%02x:00.0" % bus, "numa_node"),
           "%d\n" % (0 if g < 4 else 1))
    _w(os.path.join(root, "devices", "system", "node", "node0", "cpulist"), "0-63,128-191\n")
    _w(os.path.join(root, "devices", "system", "node", "node1", "cpulist"), "64-127,192-255\n")
    return root


def test_parse_cpulist():
    assert A.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert A.parse_cpulist("5") == [5]
    assert A.parse_cpulist("") == []


def test_agents_in_hip_order_and_bus_ids(sysfs):
    ag = A.gpu_agents(sysfs)
    assert [k for k, _ in ag] == list(range(2, 10))
    assert [b for _, b in ag] == ["0000:%02x:00.0" % b for b in BUSES]


def test_rank_to_node_and_cpus(sysfs):
    allowed = set(range(256))
    for r in range(8):
        p = A.plan_binding(r, 8, sysfs, env={}, allowed=allowed)
        node = 0 if r < 4 else 1
        assert p["numa_node"] == node and p["gpu_bdf"] == "0000:%02x:00.0" % BUSES[r]
        assert p["cpus"] == A.parse_cpulist("0-63,128-191" if node == 0 else "64-127,192-255")
        assert p["ranks_on_node"] == 4 and p["host_threads"] == 16  # 128 CPUs / 4 ranks, capped at 16


def test_visibility_variables_remap_ranks(sysfs):
    # ROCR narrows to GPUs 4..7, HIP_VISIBLE_DEVICES then picks the 3rd and 1st of those
    env = {"ROCR_VISIBLE_DEVICES": "4,5,6,7", "HIP_VISIBLE_DEVICES": "2,0"}
    assert A.gpu_numa_node(0, sysfs, env) == ("0000:%02x:00.0" % BUSES[6], 1)
    assert A.gpu_numa_node(1, sysfs, env) == ("0000:%02x:00.0" % BUSES[4], 1)
    assert A.gpu_numa_node(2, sysfs, env) is None  # only two visible
    assert A.gpu_numa_node(0, sysfs, {"CUDA_VISIBLE_DEVICES": "GPU-1234"}) is None  # UUIDs: not resolved


def test_cgroup_share_and_rehearsal(sysfs):
    # a 16-CPU share on node 1 only: rank 0 (GPU 0, node 0) has no usable CPU there -> no binding
    share = set(range(64, 80))
    assert A.plan_binding(0, 1, sysfs, env={}, allowed=share) is None
    p = A.plan_binding(4, 8, sysfs, env={}, allowed=share)
    assert p["cpus"] == list(range(64, 80)) and p["host_threads"] == 4  # 16 CPUs / 4 ranks on node 1
    # a gloo rehearsal: 2 ranks on one visible GPU share its node's CPUs
    p = A.plan_binding(0, 2, sysfs, env={"HIP_VISIBLE_DEVICES": "1"}, allowed=set(range(256)), ndev=1)
    assert p["ranks_on_node"] == 2 and p["host_threads"] == 16 and p["numa_node"] == 0


def test_missing_topology_binds_nothing(tmp_path, monkeypatch):
    assert A.plan_binding(0, 1, str(tmp_path), env={}) is None
    monkeypatch.setattr(A, "plan_binding", lambda *a, **k: None)
    before = os.sched_getaffinity(0)
    r = A.bind_rank(0, 1)
    assert r["bound"] is False and os.sched_getaffinity(0) == before


def test_visible_gpu_count_without_hip(sysfs):
    """The device count dist_setup binds with comes from the KFD topology and the visibility
    variables, so no torch.cuda call (which starts the HIP runtime's threads) precedes the binding."""
    assert A.visible_gpu_count(sysfs, env={}) == 8
    assert A.visible_gpu_count(sysfs, env={"HIP_VISIBLE_DEVICES": "2,5"}) == 2
    assert A.visible_gpu_count(sysfs, env={"ROCR_VISIBLE_DEVICES": "0,1,2,3", "CUDA_VISIBLE_DEVICES": "1"}) == 1
    assert A.visible_gpu_count(sysfs, env={"HIP_VISIBLE_DEVICES": "GPU-abc"}) is None
    assert A.visible_gpu_count(os.path.join(sysfs, "missing"), env={}) is None


def test_dist_setup_binds_before_any_device_call(monkeypatch):
    """launch.dist_setup: bind_rank runs before torch.cuda.device_count / set_device."""
    import torch
    from tmed import launch
    calls = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: calls.append("device_count") or 1)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls.append("set_device"))
    monkeypatch.setattr(A, "bind_rank", lambda *a, **k: calls.append("bind_rank") or {"bound": False})
    monkeypatch.setattr(A, "visible_gpu_count", lambda *a, **k: 1)
    monkeypatch.setenv("WORLD_SIZE", "1")
    launch.dist_setup()
    assert calls[0] == "bind_rank" and "device_count" not in calls


def test_cgroup_cpu_counters(tmp_path):
    """cpu.stat deltas over a timed region: CPUs in use, throttled periods and time; None without
    the file (a host outside a cgroup v2 CPU controller)."""
    f = tmp_path / "cpu.stat"
    f.write_text("usage_usec 1000000\nuser_usec 900000\nnr_periods 10\nnr_throttled 1\nthrottled_usec 5000\n")
    a = A.cgroup_cpu_stat(str(f))
    assert a["usage_usec"] == 1000000 and a["nr_throttled"] == 1
    f.write_text("usage_usec 9000000\nuser_usec 8000000\nnr_periods 15\nnr_throttled 4\nthrottled_usec 20000\n")
    d = A.cgroup_delta(a, A.cgroup_cpu_stat(str(f)), 0.5)
    assert d == {"cpus_used": 16.0, "periods": 5, "throttled_periods": 3, "throttled_ms": 15.0}
    assert A.cgroup_cpu_stat(str(tmp_path / "missing")) is None
    assert A.cgroup_delta(None, a, 1.0) is None
