#!/bin/bash
# Round-4 closing session 4: -m gpu suite, smoke and bench.py after the planning changes
# (tools/gpu_check.sh), then C3 traced.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_check.sh tests smoke bench || exit 1
grep -q "tests rc=0" gpurun_out/gpu_tests.log && grep -q "bench rc=0" gpurun_out/bench.log || exit 1
O=gpurun_out/final4
mkdir -p $O
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1
echo "c3 trace rc=$?"
