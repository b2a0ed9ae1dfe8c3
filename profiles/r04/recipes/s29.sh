#!/bin/bash
# Round-4 session 29: 2-rank gloo rehearsal of bench.py on the one-GPU box with the current seam
# (C2 + the C4 shard per rank + aggregation).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s29
mkdir -p $O
TMED_DIST_BACKEND=gloo timeout -k 20 700 python bench.py --gpus 2 > $O/bench_2ranks_gloo.log 2>&1
rc=$?; echo "2-rank rehearsal rc=$rc"; tail -c 800 $O/bench_2ranks_gloo.log
