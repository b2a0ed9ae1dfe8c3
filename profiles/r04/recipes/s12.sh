#!/bin/bash
# Round-4 session 12: deferred first-commit resolution — key-cache / commit GPU tests, then C1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_configs.py tests/test_gpu_commit.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python bench_commits.py --config c1 --reps 1000 > $O/c1.log 2>&1
rc=$?; echo "c1 rc=$rc"
python3 -c "import json; d=[json.loads(l) for l in open('$O/c1.log') if l.startswith('{')][-1]; print({p: v.get('p50_ms') for p, v in d['paths'].items()})"
