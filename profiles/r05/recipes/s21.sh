#!/bin/bash
# Round-5 session 21: the batched finish with every Z of a group loaded up front (cur) against one
# signature ahead (zall0 = -DTMED_FIN_ZALL=0): verify/keyed tests, then keyed C2 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s21
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_keycache.py tests/test_gpu_commit.py -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/gpu_tests.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=60 BENCH_ARGS="--no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh zall0 cur; rc=$?
cp gpurun_out/ab/ab.txt $O/ab.txt
for f in gpurun_out/ab/*.log; do grep -o '"finish_kernel_ms": [0-9.]*' $f | tail -1 | sed "s|^|$f |"; done | tee $O/finish_ms.txt
exit $rc
