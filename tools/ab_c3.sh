#!/bin/bash
# C3 A/B on one box: bench_commits.py --config c3 with the in-tree library ("cur") against a variant
# under tendermint-fork_amd/lib_var/c3old/ (built from an earlier commit.hip), three alternating rounds
# (the guide's rule: one box, interleaved, every round reported).  Writes gpurun_out/r06_s3/ab.txt:
# round, variant, headers/s, host plan ms, plan share, outcome mismatches.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06_s3
for r in 1 2 3; do
  for v in cur c3old; do
    lib=tendermint-fork_amd/lib/libtmed25519_hip.so
    [ $v = c3old ] && lib=tendermint-fork_amd/lib_var/c3old/libtmed25519_hip.so
    TMED_LIB=$PWD/$lib timeout -k 10 200 python -u bench_commits.py --config c3 --runs 7 > gpurun_out/r06_s3/c3_$v.$r.json 2> gpurun_out/r06_s3/c3_$v.$r.err || exit $?
    python3 - "$r" "$v" >> gpurun_out/r06_s3/ab.txt <<'PY'
import json, sys
r, v = sys.argv[1], sys.argv[2]
d = json.loads(open("gpurun_out/r06_s3/c3_%s.%s.json" % (v, r)).read().strip().split("\n")[-1])
x = d["direct"]
print(r, v, x["headers_per_s"], x["phase_share"]["plan_host_ms"], x["phase_share"]["plan_frac"], x["outcome_mismatches"])
PY
    tail -1 gpurun_out/r06_s3/ab.txt
  done
done
