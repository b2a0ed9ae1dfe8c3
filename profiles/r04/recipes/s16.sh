#!/bin/bash
# Round-4 session 16: -m gpu suite after the positional address check, then C3 traced and timed.
# Any failing step ends the session (no GPU step after a fault, abort or timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s16
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1
rc=$?; echo "c3 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_commits.py --config c3 --runs 7 > $O/c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=[json.loads(l) for l in open('$O/c3.log') if l.startswith('{')][-1]; print(d['value'], d['direct']['seconds_median'], d['direct']['phase_share'])"
