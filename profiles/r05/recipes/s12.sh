#!/bin/bash
# Round-5 session 12: the key-cached -A comb at radix 2^12 (21 rows) against radix 2^11 (comba11):
# the key-cache / product-default tests, keyed C2 A/B, then C3 + C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s12
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_btables.py tests/test_gpu_keycache.py tests/test_gpu_product_default.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/gpu_tests.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=60 BENCH_ARGS="--no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh comba11 cur; rc=$?
cp gpurun_out/ab/ab.txt $O/ab.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python bench_commits.py --config c3,c4 --runs 5 --blocks 12500 > $O/commits.log 2>&1; rc=$?
echo "commits rc=$rc"
exit $rc
