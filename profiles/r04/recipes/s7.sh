#!/bin/bash
# Round-4 session 7: blocksync window stream (submit/wait) — full -m gpu suite, C4 (stream + per-window), probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench_commits.py --config c4 --blocks 12500 --no-cpu > $O/c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -c 2500 $O/c4.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 120 python tools/probe_valu.py > $O/valu_rates.json 2>&1
echo "probe rc=$?"
