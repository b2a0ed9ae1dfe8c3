"""The multi-GPU path's collectives over RCCL, on the one GPU a box has: a one-rank
"nccl" process group (RCCL on ROCm) running exactly the collectives bench.py and bench_commits.py
issue at N ranks — the C2 barrier, MAX of the timed seconds (float64) and int64 tally all-reduce;
C4's aggregate_blocksync (int64 all-reduce, float64 MAX, uint8 bitmap and float64 all-gathers);
the sliced commit's int64 MIN — on device tensors.  The N-rank data movement is covered with gloo
(tests/test_dist.py, world 2 / 3 / 8); this pins the backend, dtypes and devices the driver's 8-GPU
run uses.  One child process (the process group must not outlive the test)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, os, sys
sys.path[:0] = [ROOT, os.path.join(ROOT, "tendermint-fork_amd")]
import numpy as np
import torch
import torch.distributed as dist
from tmed.dist import aggregate_blocksync
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % PORT, rank=0, world_size=1, device_id=dev)
try:
    rccl = ".".join(str(x) for x in torch.cuda.nccl.version())
except Exception as e:  # the version query only: the collectives below are the test
    rccl = "unknown (%s)" % e
out = {"backend": dist.get_backend(), "rccl": rccl}
# bench.py C2
dist.barrier()
t = torch.tensor([2.5], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
tally = torch.tensor([7, 9], dtype=torch.int64, device=dev)
dist.all_reduce(tally)
out["c2"] = [float(t.item())] + tally.tolist()
# bench_commits C4
bits = (np.arange(21) % 3 != 0).astype(np.uint8)
agg = aggregate_blocksync(bits, 21, 0, 1, verified=1234, mismatches=0, seconds=1.5, extra_max=[0.25],
                          phases=[1.0, 2.0], device=dev, per_rank=[3.0, 4.0])
out["c4"] = {"blocks_ok": agg["blocks_ok"], "blocks": agg["blocks"], "verified": agg["verified"],
             "seconds": agg["seconds"], "extra_max": agg["extra_max"], "ok_bits": agg["ok_bits"].tolist(),
             "phases": agg["phases"], "per_rank": agg["per_rank"], "bits_in": bits.tolist()}
# verify_commit_sliced's agreement on the first failing candidate
f = torch.tensor([5], dtype=torch.int64, device=dev)
dist.all_reduce(f, op=dist.ReduceOp.MIN)
out["min"] = int(f.item())
dist.barrier()
dist.destroy_process_group()
print("RESULT " + json.dumps(out), flush=True)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_one_rank_rccl_group_runs_the_benches_collectives():
    code = SCRIPT.replace("ROOT", repr(ROOT)).replace("PORT", str(_free_port()))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
    assert line, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(line[-1][len("RESULT "):])
    print(r["backend"], "RCCL", r["rccl"])
    assert r["backend"] == "nccl"
    assert r["c2"] == [2.5, 7, 9]
    c4 = r["c4"]
    assert c4["ok_bits"] == c4["bits_in"] and c4["blocks_ok"] == sum(c4["bits_in"]) and c4["blocks"] == 21
    assert c4["verified"] == 1234 and c4["seconds"] == 1.5 and c4["extra_max"] == [0.25]
    assert c4["phases"] == [[1.0, 2.0, 1.5]] and c4["per_rank"] == [[3.0, 4.0]]
    assert r["min"] == 5
