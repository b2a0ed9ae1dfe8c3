#!/bin/bash
# Round-4 session 4: full -m gpu suite, then bench (C2/C1/C3/C4/C5/ZIP).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c4 --blocks 3000 --no-cpu > $O/c4_trace.log 2>&1
echo "c4 trace rc=$?"
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1
echo "c3 trace rc=$?"
