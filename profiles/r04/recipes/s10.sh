#!/bin/bash
# Round-4 session 10: keyed device batches split over two kernel lanes — keyed GPU tests, then the
# keyed C2 A/B (TMED_LANES=1: one lane), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_btables.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2 3; do
  for L in 2 1; do
    TMED_LANES=$L timeout -k 10 120 python profiles/r04/recipes/ab_keyed.py >> $O/ab_keyed_lanes.jsonl 2>> $O/ab_keyed.err || { echo "ab failed rc=$?"; exit 1; }
  done
done
cat $O/ab_keyed_lanes.jsonl
