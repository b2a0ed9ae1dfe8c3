#!/bin/bash
# GPU suite, then an interleaved A/B of the HEAD build against the working tree (tools/ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2h
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
ROUNDS=${ROUNDS:-3} bash tools/ab.sh ${AB_VARIANTS:-head cur}
