#!/bin/bash
# Round 5 s45: the full -m gpu suite three times in a row on one box (the flake of s27 showed in one
# such run); each run in one process, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/s45
for r in 1 2 3; do
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > gpurun_out/s45/suite_$r.log 2>&1 || { echo "run $r rc=$?"; exit 1; }
  echo "run $r: $(tail -n 1 gpurun_out/s45/suite_$r.log)"
done
