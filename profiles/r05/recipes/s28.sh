#!/bin/bash
# Round 5 s28: the pipelined seam's merge race (Group::add_run read the next part's first offset).
# 1. the skew regression test against the library built with the old add_run (expected: it fails);
# 2. the same test, the C3 many-sets tests and the pipelined-seam tests on the fixed library;
# 3. tools/stress/c3_stress.py, 700 generic calls (before the fix: 3 of 700 with mismatches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
TMED_LIB=$PWD/tendermint-fork_amd/lib_var/oldrun/libtmed25519_hip.so timeout -k 10 300 $T -m gpu \
  tests/test_gpu_configs.py -k merged_out_of_order > gpurun_out/s28_oldlib.log 2>&1
rc=$?; echo "old library rc=$rc (1 expected)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 $T -m gpu tests/test_gpu_configs.py -k "merged_out_of_order or many_sets" \
  tests/test_gpu_commit.py > gpurun_out/s28_fixed.log 2>&1 || { echo "fixed tests rc=$?"; exit 1; }
echo "fixed tests ok"
timeout -k 10 300 python -u tools/stress/c3_stress.py 700 70000 > gpurun_out/s28_stress.log 2>&1
echo "stress rc=$?"
