#!/bin/bash
# Round-5 session 23: the key-cached main kernel with each comb row fetched two additions ahead into
# LDS (TMED_KS_LDS2=1, cur) against one row ahead in registers (lds0): keyed tests, then keyed C2
# (bench.py) and C4 (bench_commits.py) alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s23
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_keychunks.py tests/test_gpu_keycache.py tests/test_gpu_btables.py -x -v --timeout 250 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/tests.log; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab/ab.txt
ROUNDS=3 STEPS=60 BENCH_ARGS="--no-c4 --no-c3 --no-c5 --no-zip215" bash tools/ab.sh lds0 cur; rc=$?
cp gpurun_out/ab/ab.txt $O/ab.txt
for f in gpurun_out/ab/*.log; do grep -o '"c2_keyset_variant".\{0,400\}' $f | grep -o '"kernel_avg_ms": [0-9.]*' | head -1 | sed "s|^|$f |"; done | tee $O/keyed_main_ms.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in lds0 cur; do
    lib=tendermint-fork_amd/lib/libtmed25519_hip.so
    [ $v = cur ] || lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so
    TMED_LIB=$lib timeout -k 10 400 python bench_commits.py --config c4 --blocks 12500 > $O/c4_$v.$r.log 2>&1; rc=$?
    echo "$r $v rc=$rc $(grep '^{' $O/c4_$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C4", round(d["value"]), "mismatches", d["outcome_mismatches"])')" | tee -a $O/c4_ab.txt
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
exit 0
