#!/bin/bash
# Round-4 session 18: host pool wake-up cost against polling time (TMED_POOL_SPIN_US), probe and
# C3 A/B alternating (0 = the current policy).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s18
mkdir -p $O
for sp in 0 300 2000; do
  TMED_POOL_SPIN_US=$sp timeout -k 5 60 ./tools/pool_probe > $O/pool_probe_spin$sp.jsonl 2>&1 || exit 1
done
echo "probes ok"; grep -h "gap100\"" $O/pool_probe_spin*.jsonl
for rep in 1 2; do
  for sp in 0 300 2000; do
    TMED_POOL_SPIN_US=$sp timeout -k 10 300 python bench_commits.py --config c3 --runs 5 > $O/c3_spin${sp}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c3 spin $sp rc=$rc"; exit $rc; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/c3_spin${sp}_$rep.log') if l.startswith('{')][-1]; print('spin', $sp, d['value'], d['direct']['seconds_median'], d['direct']['phase_share'])"
  done
done
