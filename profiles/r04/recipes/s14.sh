#!/bin/bash
# Round-4 session 14: generic C2 batch split over two kernel lanes — verify GPU tests, then C2 A/B
# (TMED_LANES=1: one lane), alternating; C4 with the 4-window stream chunks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s14
mkdir -p $O
for r in 1 2 3; do
  for L in 2 1; do
    TMED_LANES=$L timeout -k 10 200 python bench.py --no-c1 --no-c3 --no-c4 --no-c5 --no-zip215 --no-keyset --no-cpu-baseline --steps 100 > $O/c2_lanes$L.$r.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "c2 rc=$rc"; exit $rc;; esac
    python3 -c "import json; d=[json.loads(l) for l in open('$O/c2_lanes$L.$r.log') if l.startswith('{')][-1]; print('lanes=$L', d['value'], d['ms_per_step'], d['all_valid'])"
  done
done
timeout -k 10 300 python bench_commits.py --config c4 --blocks 12500 --no-cpu > $O/c4.log 2>&1
echo "c4 rc=$?"; python3 -c "import json; d=[json.loads(l) for l in open('$O/c4.log') if l.startswith('{')][-1]; print(d['value'], d['per_window_calls']['value'], d['outcome_mismatches'])"
