#!/bin/bash
# Round-5 session 19: key combs in chunks of 512 keys (no copy / free when a key set grows): the
# full -m gpu suite (incl. test_gpu_keychunks.py), C4 + C3 twice (C3's second call is where the
# pool grows past C4's keys), then bench.py's default run (wall time, C3 second call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s19
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/tests.log; tail -3 $O/tests.log
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  t0=$(date +%s)
  timeout -k 10 600 python bench_commits.py --config c4,c3 --runs 5 --blocks 12500 > $O/commits.$r.log 2>&1; rc=$?
  echo "$r rc=$rc wall=$(( $(date +%s) - t0 ))s $(grep '^{' $O/commits.$r.log | python3 -c 'import json,sys
out=[]
for l in sys.stdin:
  d=json.loads(l)
  out.append(("C3 %.0f second_call %.3f s pool %d" % (d["direct"]["headers_per_s"], d["direct"]["second_call_seconds"], d["direct"]["pool_keys"])) if "direct" in d else ("C4 %.0f" % d["value"]))
print(" ".join(out))')" | tee -a $O/ab.txt
  case $rc in 0) ;; *) exit $rc;; esac
done
t0=$(date +%s); timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench wall $(( $(date +%s) - t0 )) s rc=$rc" | tee -a $O/bench.log
exit $rc
