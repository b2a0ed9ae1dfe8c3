#!/bin/bash
# Round 5 s32: the generic throughput kernels (prep, prep_r, half-size main) in blocks of 64 / 128
# threads against 256 (TMED_HS_BLOCK): C2 legs alternating on one box, then the verify tests on 64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=30 BENCH_ARGS="--no-keyset --no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh cur hs64 hs128 || exit $?
TMED_LIB=$PWD/tendermint-fork_amd/lib_var/hs64/libtmed25519_hip.so timeout -k 10 400 python -u -m pytest -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_verify.py tests/test_gpu_btables.py \
  tests/test_gpu_zip215.py > gpurun_out/s32_tests_hs64.log 2>&1
echo "hs64 tests rc=$?"
