#!/bin/bash
# Round 5 s29: the seam tests under host-pool scheduling jitter (tests/test_gpu_jitter.py):
# 1. against the library built with the old Group::add_run (does jitter alone expose that race?);
# 2. on the current library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
TMED_LIB=$PWD/tendermint-fork_amd/lib_var/oldrun/libtmed25519_hip.so timeout -k 10 400 $T -m gpu \
  tests/test_gpu_jitter.py > gpurun_out/s29_oldlib.log 2>&1
rc=$?; echo "old library rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 $T -x -m gpu tests/test_gpu_jitter.py > gpurun_out/s29_jitter.log 2>&1
echo "current library rc=$?"
