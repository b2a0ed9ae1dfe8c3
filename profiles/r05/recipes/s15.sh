#!/bin/bash
# Round-5 session 15: both key combs (radix 256 for the latency kernels, radix 2^12 for the
# throughput kernel) built in runs with one batched inversion per run: the full -m gpu suite,
# C1, and a kernel trace of the keyed C2 leg (comb_fill / comba_fill times).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s15
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/gpu_tests.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench_commits.py --config c1 > $O/c1.log 2>&1; rc=$?
echo "c1 rc=$rc"; grep '^{' $O/c1.log | cut -c1-400
case $rc in 124|134|137|139) exit $rc;; esac
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --no-cpu-baseline --no-c4 --no-c5 --no-zip215 > $R/$O/bench.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
