#!/bin/bash
# Round-4 session 8: C3 host work (set_hash, shared templates, parallel checks/merge, prefetch) —
# C3-shaped GPU tests, C3 bench + trace, VALU probes, then the 2-rank gloo rehearsal of bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_configs.py tests/test_gpu_commit.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python bench_commits.py --config c3 --runs 7 > $O/c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -c 1200 $O/c3.log
case $rc in 0) ;; *) exit $rc;; esac
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 2 > $O/c3_trace.log 2>&1
echo "c3 trace rc=$?"
timeout -k 10 120 python tools/probe_valu.py > $O/valu_rates.json 2>&1
echo "probe rc=$?"
# keyed C2 A/B: old batched finish / pipelined finish (default) / + 4-wave keyed prep
for r in 1 2 3; do
  for L in tendermint-fork_amd/lib/ab/libtmed_finold.so tendermint-fork_amd/lib/libtmed25519_hip.so tendermint-fork_amd/lib/ab/libtmed_prep4.so; do
    TMED_LIB=$PWD/$L timeout -k 10 120 python profiles/r04/recipes/ab_keyed.py >> $O/ab_keyed.jsonl 2>> $O/ab_keyed.err || { echo "ab failed rc=$?"; exit 1; }
  done
done
cat $O/ab_keyed.jsonl
TMED_DIST_BACKEND=gloo timeout -k 20 700 python bench.py --gpus 2 > $O/bench_2ranks_gloo.log 2>&1
rc=$?; echo "2-rank rehearsal rc=$rc"; tail -c 600 $O/bench_2ranks_gloo.log
