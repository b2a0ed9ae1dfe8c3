#!/bin/bash
# Round-4 session 24: C3 on one box, the library at the start of this session's host work
# (lib/ab/libtmed_s14.so, commit bd046c2) against the current one, alternating, three runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s24
mkdir -p $O
for rep in 1 2 3; do
  for L in tendermint-fork_amd/lib/ab/libtmed_s14.so tendermint-fork_amd/lib/libtmed25519_hip.so; do
    tag=$(basename $L .so)
    TMED_LIB=$PWD/$L timeout -k 10 300 python bench_commits.py --config c3 --runs 5 > $O/c3_${tag}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c3 $tag rc=$rc"; exit $rc; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/c3_${tag}_$rep.log') if l.startswith('{')][-1]; print('$tag', d['value'], d['direct']['seconds_median'], d['direct']['phase_share']['plan_frac'], d['direct']['all_ok'], d['bisection']['headers_per_s'])"
  done
done
