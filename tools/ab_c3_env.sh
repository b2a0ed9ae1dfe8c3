#!/bin/bash
# C3 A/B of env settings on one box: bench_commits.py --config c3, each variant of VARIANTS ('|'
# separated, e.g. "TMED_HOST_THREADS=16|TMED_HOST_THREADS=12") once per round, ROUNDS alternating
# rounds.  Writes $OUT/ab.txt: round, variant, headers/s, host plan ms, plan share, outcome
# mismatches, then the cgroup's CPU counters over the timed calls (CPUs in use, periods, throttled
# periods, throttled ms).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/c3_env}
mkdir -p $OUT
cat /sys/fs/cgroup/cpu.max > $OUT/cpu_max.txt 2>&1 || true
IFS='|' read -ra VLIST <<< "${VARIANTS:-TMED_HOST_THREADS=16|TMED_HOST_THREADS=12}"
for r in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for cfg in "${VLIST[@]}"; do
    i=$((i + 1))
    env $cfg timeout -k 10 200 python -u bench_commits.py --config c3 --runs 7 > $OUT/c3_v$i.$r.json 2> $OUT/c3_v$i.$r.err || exit $?
    python3 - "$r" "$cfg" "$OUT/c3_v$i.$r.json" >> $OUT/ab.txt <<'PY'
import json, sys
r, v, f = sys.argv[1:4]
d = json.loads(open(f).read().strip().split("\n")[-1])
x = d["direct"]
p = x["phase_share"]
cg = p.get("host_cgroup") or {}
print(r, v, x["headers_per_s"], p["plan_host_ms"], p["plan_frac"], x["outcome_mismatches"],
      cg.get("cpus_used"), cg.get("periods"), cg.get("throttled_periods"), cg.get("throttled_ms"))
PY
    tail -1 $OUT/ab.txt
  done
done
