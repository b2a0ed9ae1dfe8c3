#!/bin/bash
# A/B of library builds on the key-cached C2 variant (bench.py's c2_keyset leg).  Usage:
# tools/ab_keyset.sh NAME... (lib_var/NAME or "cur"); ROUNDS (default 3).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/abk
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "$@"; do
    if [ "$v" = cur ]; then lib=tendermint-fork_amd/lib/libtmed25519_hip.so; else lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so; fi
    TMED_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --no-c1 --no-peak > $OUT/$v.$r.log 2>&1; rc=$?
    line=$(tail -1 $OUT/$v.$r.log)
    echo "$r $v rc=$rc $(echo "$line" | python3 -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); k=d["c2_keyset_variant"]
  print("keyed", k["value"], k["all_valid"], "main", k["roofline"]["kernel_avg_ms"], "prep", k["roofline"]["prep_kernel_ms"], "| generic", d["value"])
except Exception as e: print("parse-fail", e)')" | tee -a $OUT/abk.txt
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
