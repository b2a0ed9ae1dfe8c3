#!/bin/bash
# Round-5 session 9: cost of the lattice step inside prep_r (nolat: every lane takes the (k, 1)
# fallback — correct decisions, W = 64, prep timing only) and the keyed finish at 131,072 lanes
# (8 signatures per inversion) against 65,536 (16).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s9
mkdir -p $O
rm -f gpurun_out/ab/ab.txt
ROUNDS=2 STEPS=40 BENCH_ARGS="--no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh cur nolat fin128k; rc=$?
cp gpurun_out/ab/ab.txt $O/ab.txt
exit $rc
