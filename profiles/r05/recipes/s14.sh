#!/bin/bash
# Round-5 session 14: the radix-2^12 comb built in runs of 8 entries per lane with one batched
# inversion per run (was: double-and-add + an inversion per entry, 1.6 s for 10k keys): key-cache
# tests, then C3 / C4 and a kernel trace of the keyed C2 leg (comba_fill time).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s14
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_btables.py tests/test_gpu_keycache.py tests/test_gpu_product_default.py tests/test_gpu_configs.py tests/test_gpu_commit.py -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/gpu_tests.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench_commits.py --config c3,c4 --runs 5 --blocks 12500 > $O/commits.log 2>&1; rc=$?
echo "commits rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --no-cpu-baseline --no-c1 --no-c3 --no-c4 --no-c5 --no-zip215 > $R/$O/bench_keyed.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
