#!/bin/bash
# Round-5 session 6: C2 generic + keyed A/B of the SHA-512 first-pass peel: "cur" (peeled),
# "sha0" (TMED_SHA_PEEL=0), "base" (the session-start kernels), alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s6
mkdir -p $O
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=60 BENCH_ARGS="--no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh base cur sha0; rc=$?
cp gpurun_out/ab/ab.txt $O/ab.txt
exit $rc
