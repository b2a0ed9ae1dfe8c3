#!/bin/bash
# Round-4 session 11: C1 first-call trace (key-cache resolution on a miss), then the rocprofv3
# kernel-trace summary of bench.py and the PMC passes (tools/gpu_check.sh prof pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s11
mkdir -p $O
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c1 --reps 100 --no-cpu > $O/c1_trace.log 2>&1
echo "c1 trace rc=$?"
bash tools/gpu_check.sh prof pmc
