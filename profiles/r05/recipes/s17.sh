#!/bin/bash
# Round-5 session 17: the batched finish's group size by ceiling (at most 65,536 lanes: one
# latency-bound wave per SIMD) against the floor (finfloor), C3 + C4 alternating; then the 2-rank
# gloo rehearsal of bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s17
mkdir -p $O
for r in 1 2 3; do
  for v in finfloor cur; do
    lib=tendermint-fork_amd/lib/libtmed25519_hip.so
    [ $v = cur ] || lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so
    TMED_LIB=$lib timeout -k 10 600 python bench_commits.py --config c3,c4 --runs 5 --blocks 12500 > $O/$v.$r.log 2>&1; rc=$?
    echo "$r $v rc=$rc $(grep '^{' $O/$v.$r.log | python3 -c 'import json,sys
out=[]
for l in sys.stdin:
  d=json.loads(l)
  out.append(("C3 %.0f" % d["direct"]["headers_per_s"]) if "direct" in d else ("C4 %.0f" % d["value"]))
print(" ".join(out))')" | tee -a $O/ab.txt
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
bash profiles/r05/recipes/s16.sh; rc=$?
cp -r gpurun_out/r05s16 $O/ 2>/dev/null
exit $rc
