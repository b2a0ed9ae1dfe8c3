#!/bin/bash
# Round 5 s33: the half-size hand-off placed long waves first (TMED_HS_LONG_FIRST=1) against short
# first: C2 alternating on one box, then the verify tests on the variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
rm -f gpurun_out/ab/ab.txt
ROUNDS=${ROUNDS:-4} STEPS=30 BENCH_ARGS="--no-keyset --no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh cur lf || exit $?
TMED_LIB=$PWD/tendermint-fork_amd/lib_var/lf/libtmed25519_hip.so timeout -k 10 400 python -u -m pytest -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_verify.py tests/test_gpu_btables.py \
  tests/test_gpu_zip215.py > gpurun_out/s33_tests_lf.log 2>&1
echo "lf tests rc=$?"
