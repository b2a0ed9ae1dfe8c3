#!/bin/bash
# Round-4 session 1: key-set cache GPU tests, the full -m gpu suite, the C4 trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=gpurun_out/s1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_zip215.py::test_dense_failures_cut_off -x -v --timeout 200 --timeout-method thread > $O/kc_tests.log 2>&1
rc=$?; echo "kc tests rc=$rc"; tail -3 $O/kc_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
bash profiles/r04/recipes/c4_trace.sh
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.log
