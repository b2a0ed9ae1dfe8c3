#!/bin/bash
# Round-5 session 10: Lehmer rounds in the lattice step (verify_hs.h hs_lehmer_round) against the
# one-step loop (nolehmer = -DTMED_LEHMER=0): the verify tests, then C2 A/B (prep_kernels_ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/gpu_tests.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=40 BENCH_ARGS="--no-keyset --no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh nolehmer cur; rc=$?
cp gpurun_out/ab/ab.txt $O/ab.txt
exit $rc
