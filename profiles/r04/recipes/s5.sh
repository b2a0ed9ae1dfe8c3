#!/bin/bash
# Round-4 session 5: C3 candidate aliasing — C3-shaped GPU tests, then C3 bench (plain, traced).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_keycache.py tests/test_gpu_commit.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -c 1500 $O/c3.log
case $rc in 0) ;; *) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 2 > $O/c3_trace.log 2>&1
echo "c3 trace rc=$?"
