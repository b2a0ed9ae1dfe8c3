#!/bin/bash
# Round-5 session 2: cache policy of the main kernel's memory streams (TMED_SLAB_NT variants) and the
# global-address-space identity row ("cur") against the round-4 kernels ("base"); alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=60 BENCH_ARGS="--no-keyset --no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh base cur nt1 nt2 nt4 nt7
rc=$?
mkdir -p gpurun_out/r05s2 && cp gpurun_out/ab/ab.txt gpurun_out/r05s2/
exit $rc
