#!/bin/bash
# Round-5 session 1: the product-default (cache-on) tests and the changed seam teardown, then bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_product_default.py tests/test_gpu_configs.py tests/test_gpu_keycache.py tests/test_gpu_concurrency.py \
  > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc" | tee -a $O/bench.log
exit $rc
