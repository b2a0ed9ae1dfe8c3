#!/bin/bash
# Full GPU suite, the default bench line, and the generic latency/throughput crossover sweep.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --steps 20 > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_avg_ms"], d["roofline"]["prep_kernels_ms"], json.dumps(d["c1_verifycommit_p50"])[:600])'
for m in 0 65536; do
  TMED_GLAT_MAX=$m timeout -k 10 300 python3 tools/lat_probe.py 175 4096 8192 16384 32768 65536 > $OUT/sweep_glat$m.jsonl 2>&1 || exit $?
done
cat $OUT/sweep_glat*.jsonl
