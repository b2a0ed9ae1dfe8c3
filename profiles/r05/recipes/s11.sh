#!/bin/bash
# Round-5 session 11: C4 with the shim's flatten overlapped with the device (value_incl_marshal_overlapped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s11
mkdir -p $O
timeout -k 10 600 python bench_commits.py --config c4 --blocks 12500 > $O/c4.log 2>&1; rc=$?
echo "c4 rc=$rc"; grep '^{' $O/c4.log | python3 -c 'import json,sys
for l in sys.stdin:
  d=json.loads(l); print({k: d.get(k) for k in ("value","value_incl_marshal","value_incl_marshal_overlapped","marshal_seconds_max_rank","seconds","outcome_mismatches")})'
exit $rc
