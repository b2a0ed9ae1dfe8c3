#!/bin/bash
# Round-5 session 3: C3 and C4 with the compiled shim marshal (shim/go_marshal.cpp) beside the seam.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s3
mkdir -p $O
timeout -k 10 600 python bench_commits.py --config c3,c4 --runs 5 --blocks 12500 > $O/commits.log 2>&1; rc=$?
echo "commits rc=$rc" | tee -a $O/commits.log
exit $rc
