#!/bin/bash
# Round-4 session 31: keyed C2 with the batched finish over 131,072 / 262,144 lanes (8 / 4
# signatures per lane, 2 / 4 waves per SIMD) against 65,536 (16 per lane, one wave), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s31
mkdir -p $O
for rep in 1 2 3; do
  for L in tendermint-fork_amd/lib/libtmed25519_hip.so tendermint-fork_amd/lib/ab/libtmed_fin131k.so tendermint-fork_amd/lib/ab/libtmed_fin262k.so; do
    TMED_LIB=$PWD/$L timeout -k 10 200 python profiles/r04/recipes/ab_keyed.py >> $O/ab_keyed.jsonl 2>> $O/ab_keyed.err
    rc=$?; [ $rc -eq 0 ] || { echo "ab rc=$rc"; exit $rc; }
  done
done
cat $O/ab_keyed.jsonl
