#!/bin/bash
# Round-4 session 2: full -m gpu suite, bench, C3 with the seam trace, C4 timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench.log
case $rc in 124|134|137|139) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1
rc=$?; echo "c3 trace rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/c4prof -o run --output-format csv -- python3 $R/bench_commits.py --config c4 --blocks 3000 --no-cpu > $R/$O/c4.log 2>&1
echo "c4 trace rc=$?"
