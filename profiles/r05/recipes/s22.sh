#!/bin/bash
# Round-5 session 22: 2-rank gloo rehearsal of bench.py with the current library (key combs in 512-key
# chunks, the warmed-set C1 path; C4's overlapped-marshal pass off at world > 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s22
mkdir -p $O
TMED_DIST_BACKEND=gloo timeout -k 10 700 python bench.py --gpus 2 --steps 20 --c4-blocks 4000 --no-cpu-baseline > $O/rehearsal_gloo2.log 2>&1; rc=$?
echo "rehearsal rc=$rc"; tail -c 400 $O/rehearsal_gloo2.log
exit $rc
