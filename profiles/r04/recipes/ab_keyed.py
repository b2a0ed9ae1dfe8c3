"""A/B of the keyed C2 step (bench.py c2_keyset) for the library named by TMED_LIB: one JSON line
with verifies/s and the prep / main / finish kernel times (2^20 signatures, 10k keys)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tendermint-fork_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from tmed import Engine  # noqa: E402

dev = torch.device("cuda", 0)
eng = Engine(0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
r = bench.c2_keyset(eng, dev, s, 1 << 20, 20, 3, None)
rf = r["roofline"]
print(json.dumps({"lib": os.environ.get("TMED_LIB", "default"), "lanes": os.environ.get("TMED_LANES", "2"),
                  "value": r["value"], "all_valid": r["all_valid"],
                  "prep_ms": rf["prep_kernel_ms"], "main_ms": rf["kernel_avg_ms"] * rf["launches_per_step"],
                  "finish_ms": rf["finish_kernel_ms"]}), flush=True)
eng.close()
