#!/bin/bash
# Round-4 session 22: keyed prep at 4 waves/SIMD (128 VGPRs, 4 spilled) against 3 (130 VGPRs),
# keyed C2 A/B alternating, three runs each (profiles/r04/recipes/ab_keyed.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s22
mkdir -p $O
for rep in 1 2 3; do
  for L in tendermint-fork_amd/lib/libtmed25519_hip.so tendermint-fork_amd/lib/ab/libtmed_ksprep4.so; do
    TMED_LIB=$PWD/$L timeout -k 10 200 python profiles/r04/recipes/ab_keyed.py >> $O/ab_keyed.jsonl 2>> $O/ab_keyed.err
    rc=$?; [ $rc -eq 0 ] || { echo "ab rc=$rc"; exit $rc; }
  done
done
cat $O/ab_keyed.jsonl
