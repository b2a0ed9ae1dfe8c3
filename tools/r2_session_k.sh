#!/bin/bash
# Secondary configs on the current build: C5 adversarial mix, C3/C4 through the seam, key-cached C2.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2k
mkdir -p $OUT
timeout -k 10 600 python bench.py --mix c5 --no-c1 --no-keyset > $OUT/bench_c5.log 2>&1 || exit $?
grep '^{' $OUT/bench_c5.log | cut -c1-200
timeout -k 10 900 python bench_commits.py --config c3,c4 > $OUT/bench_commits.log 2>&1 || exit $?
grep '^{' $OUT/bench_commits.log | cut -c1-400
timeout -k 10 300 python bench_keyset.py > $OUT/bench_keyset.log 2>&1 || exit $?
grep '^{' $OUT/bench_keyset.log | cut -c1-300
