#!/bin/bash
# C1 latency A/B of library variants: bench_commits c1 (generic + keyed p50) and the latency
# kernels' device times at n = 175 (tools/lat_probe.py), interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2j
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-cur}; do
    if [ "$v" = cur ]; then lib=tendermint-fork_amd/lib/libtmed25519_hip.so; else lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so; fi
    TMED_LIB=$lib timeout -k 10 300 python bench_commits.py --config c1 --reps ${REPS:-500} > $OUT/c1_$v.$r.log 2>&1 || exit $?
    TMED_LIB=$lib timeout -k 10 120 python tools/lat_probe.py 175 > $OUT/lat_$v.$r.log 2>&1 || exit $?
    echo "$r $v $(grep '^{' $OUT/c1_$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps(d.get("paths")))') $(grep '^{' $OUT/lat_$v.$r.log)"
  done
done
