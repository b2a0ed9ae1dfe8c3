"""C1 phase breakdown (tools only): the seam's host plan / verify (staging + device + wait) /
replay wall times (tmed_seam_phase_us) and the per-group trace (TMED_TRACE=1 on stderr: templates,
stage, device, scatter) over repeated 175-validator VerifyCommit calls, generic and key-cached."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tendermint-fork_amd"))


def main():
    import bench_commits as B
    import tmed.types as T
    from tmed import Engine, lib
    from tmed.workload import make_valset, pubkeys_of, seeds_from_tag, sign_commits
    eng = Engine(0)
    l = lib()
    l.tmed_seam_phase_us.argtypes = [ctypes.POINTER(ctypes.c_double)]
    n = 175
    seeds = seeds_from_tag(b"tmed-bench-key", 0, n)
    pubs = pubkeys_of(eng, seeds)
    vals, order = make_valset(pubs, [10] * n)
    addrs = np.array([np.frombuffer(v.address, np.uint8) for v in vals.validators])
    bid = B.block_id(b"tmed-c1")
    commit = sign_commits(eng, "test_chain_id", [(seeds[order], addrs, 3, 0, bid, B.T2023, None)])[0]
    for path in ("generic", "keyset"):
        if path == "keyset":
            vals.keyset = eng.keyset_load(np.array([np.frombuffer(v.pub_key, np.uint8) for v in vals.validators]))
        pb = T.PreparedBatch([(T.MODE_COMMIT, vals, "test_chain_id", bid, 3, commit, 0, 0)])
        for _ in range(20):
            pb.run(eng)
        ph, wall = [], []
        buf = (ctypes.c_double * 3)()
        for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 300):
            t0 = time.perf_counter()
            pb.run(eng)
            wall.append((time.perf_counter() - t0) * 1e6)
            l.tmed_seam_phase_us(buf)
            ph.append(list(buf))
        ph = np.median(np.array(ph), axis=0)
        print(json.dumps({"path": path, "wall_p50_us": round(float(np.median(wall)), 1),
                          "plan_us": round(float(ph[0]), 1), "verify_us": round(float(ph[1]), 1),
                          "replay_us": round(float(ph[2]), 1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
