#!/bin/bash
# Round-4 session 13: C3 and C4 host-phase traces with the new host pool.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s13
mkdir -p $O
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1
echo "c3 trace rc=$?"
timeout -k 10 300 python bench_commits.py --config c3 --runs 7 > $O/c3.log 2>&1
echo "c3 rc=$?"; python3 -c "import json; d=[json.loads(l) for l in open('$O/c3.log') if l.startswith('{')][-1]; print(d['value'], d['direct']['seconds_median'], d['direct']['phase_share'])"
