#!/bin/bash
# Round-5 session 7: 2-rank gloo rehearsal of bench.py on the one GPU (per-rank NUMA binding and
# C4 memory mode in the JSON), then C3 traced (key-set cache compare against the pool key table).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s7
mkdir -p $O
TMED_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 --c4-blocks 4000 --no-cpu-baseline > $O/rehearsal_gloo2.log 2>&1; rc=$?
echo "rehearsal rc=$rc"; tail -c 600 $O/rehearsal_gloo2.log
case $rc in 124|134|137|139) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1; rc=$?
echo "c3 trace rc=$rc"
exit $rc
