#!/bin/bash
# Round-5 session 18: the key-set cache pool's combs grown in place (HIP virtual memory, VmmRange)
# against growth by copying (TMED_KS_VMM=0): key-cache / config / commit tests, C3 + C4 alternating
# (C3's second call is where the pool grows past C4's 10k keys), then bench.py's default run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s18
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_keycache.py tests/test_gpu_configs.py tests/test_gpu_commit.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" | tee -a $O/tests.log; tail -3 $O/tests.log
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for v in 1 0; do
    t0=$(date +%s)
    TMED_KS_VMM=$v timeout -k 10 600 python bench_commits.py --config c4,c3 --runs 5 --blocks 12500 > $O/vmm$v.$r.log 2>&1; rc=$?
    echo "$r vmm=$v rc=$rc wall=$(( $(date +%s) - t0 ))s $(grep '^{' $O/vmm$v.$r.log | python3 -c 'import json,sys
out=[]
for l in sys.stdin:
  d=json.loads(l)
  out.append(("C3 %.0f second_call %.3f s" % (d["direct"]["headers_per_s"], d["direct"]["second_call_seconds"])) if "direct" in d else ("C4 %.0f" % d["value"]))
print(" ".join(out))')" | tee -a $O/ab.txt
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
t0=$(date +%s); timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?; echo "bench wall $(( $(date +%s) - t0 )) s rc=$rc" | tee -a $O/bench.log
exit $rc
