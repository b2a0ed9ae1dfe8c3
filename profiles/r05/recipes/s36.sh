#!/bin/bash
# Round 5 s36: the pipelined seam's batch size (TMED_PIPE_SIGS) for the timed C3 call (20,000
# requests, 3.5M signatures, keyed): 2^18, 2^19 (default), 2^20 and 3x2^19, alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/s36
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${SIZES:-262144 524288 1048576 1572864}; do
    TMED_PIPE_SIGS=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-peak --no-c1 \
      --no-keyset --no-c4 --no-c5 --no-zip215 > gpurun_out/s36/$v.$r.log 2>&1; rc=$?
    case $rc in 0) ;; *) echo "$v rc=$rc"; exit $rc;; esac
    grep '^{' gpurun_out/s36/$v.$r.log | tail -1 | python3 -c 'import json,sys
d=json.loads(sys.stdin.read()); c=d["c3_light_client"]["direct"]; p=c["phase_share"]
print(sys.argv[1], sys.argv[2], c["headers_per_s"], c["seconds_median"], "plan", p["plan_frac"], "mism", c["outcome_mismatches"])' $r $v | tee -a gpurun_out/s36/ab.txt
  done
done
