#!/bin/bash
# Round-4 session 17: host fork-join cost (tools/pool_probe.cpp) on the box, and C3 with 8 host
# threads against the default 16 (how much of the light-client batch is thread-parallel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s17
mkdir -p $O
timeout -k 5 60 ./tools/pool_probe > $O/pool_probe.jsonl 2>&1; echo "probe rc=$?"; cat $O/pool_probe.jsonl
TMED_HOST_THREADS=8 timeout -k 5 60 ./tools/pool_probe > $O/pool_probe8.jsonl 2>&1; echo "probe8 rc=$?"
TMED_HOST_THREADS=8 TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_t8_trace.log 2>&1
rc=$?; echo "c3 t8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
TMED_HOST_THREADS=8 timeout -k 10 300 python bench_commits.py --config c3 --runs 5 > $O/c3_t8.log 2>&1
rc=$?; echo "c3 t8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=[json.loads(l) for l in open('$O/c3_t8.log') if l.startswith('{')][-1]; print(d['value'], d['direct']['seconds_median'], d['direct']['phase_share'])"
