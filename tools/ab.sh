#!/bin/bash
# A/B of library builds on one box: bench.py's C2 leg, interleaved rounds (rule 24 of the
# CDNA guide: one box, alternating, report every round).  Usage: tools/ab.sh NAME... where
# NAME is a directory under tendermint-fork_amd/lib_var/ holding libtmed25519_hip.so, or
# "cur" for the in-tree build, or "env:VAR=value[,VAR=value]" for the in-tree build under those settings.  ROUNDS (default 3), STEPS (default 20), BENCH_ARGS (default --no-keyset).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/ab
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    envs=""
    case $v in
      env:*) lib=tendermint-fork_amd/lib/libtmed25519_hip.so; envs=${v#env:};;  # in-tree build with VAR=value[,VAR=value]
      cur) lib=tendermint-fork_amd/lib/libtmed25519_hip.so;;
      *) lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so;;
    esac
    env ${envs//,/ } TMED_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --no-cpu-baseline --no-c1 ${BENCH_ARGS:---no-keyset} > $OUT/$v.$r.log 2>&1; rc=$?
    line=$(grep '^{' $OUT/$v.$r.log | tail -1)
    echo "$r $v rc=$rc $(echo "$line" | python3 -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); r=d["roofline"]
  k=d.get("c2_keyset_variant")
  print(d["value"], d["ms_per_step"], "main", r["kernel_avg_ms"], "prep", r["prep_kernels_ms"], "peak", r["peak"],
        *(["keyed", k["value"], k["roofline"]["kernel_avg_ms"]] if k else []))
except Exception as e: print("parse-fail", e)')" | tee -a $OUT/ab.txt
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
