#!/bin/bash
# bench (all legs) + 2-rank gloo rehearsal of bench.py's own rank spawning
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2b
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 300 $OUT/bench.log
case $rc in 124|134|137|139) exit $rc;; esac
TMED_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --sigs 262144 --no-cpu-baseline --no-c1 --no-keyset > $OUT/bench_2ranks.log 2>&1; rc=$?
echo "bench2 rc=$rc"; tail -c 300 $OUT/bench_2ranks.log
exit 0
