#!/bin/bash
# Round-4 session 3: full -m gpu suite; C4 and C3 with the seam trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c4 --blocks 3000 --no-cpu > $O/c4_trace.log 2>&1
rc=$?; echo "c4 rc=$rc"; grep '^{' $O/c4_trace.log | cut -c1-300
case $rc in 124|134|137|139) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1
rc=$?; echo "c3 rc=$rc"; grep '^{' $O/c3_trace.log | cut -c1-300
