#!/bin/bash
# Round-4 session 9: second kernel lane for keyed pipelined batches — seam GPU tests, then C4
# A/B (two lanes vs TMED_LANES=1), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_configs.py tests/test_gpu_keycache.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for L in 2 1; do
    TMED_LANES=$L timeout -k 10 300 python bench_commits.py --config c4 --blocks 12500 --no-cpu > $O/c4_lanes$L.$r.log 2>&1
    rc=$?; echo "c4 lanes=$L run $r rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
    python3 -c "import json,sys; d=[json.loads(l) for l in open('$O/c4_lanes$L.$r.log') if l.startswith('{')][-1]; print('lanes=$L', d['value'], d['per_window_calls']['value'], d['outcome_mismatches'])"
  done
done
