#!/bin/bash
# Round-4 closing session 3: -m gpu suite, smoke, bench.py, rocprofv3 kernel-trace summary
# (tools/gpu_check.sh), then C3 on the same box: the library at the start of this session's host
# work (lib/ab/libtmed_s14.so, commit bd046c2) against the current one, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_check.sh tests smoke bench prof || exit 1
grep -q "tests rc=0" gpurun_out/gpu_tests.log && grep -q "bench rc=0" gpurun_out/bench.log || exit 1
O=gpurun_out/final3
mkdir -p $O
for rep in 1 2; do
  for L in tendermint-fork_amd/lib/ab/libtmed_s14.so tendermint-fork_amd/lib/libtmed25519_hip.so; do
    tag=$(basename $L .so)
    TMED_LIB=$PWD/$L timeout -k 10 300 python bench_commits.py --config c3 --runs 5 > $O/c3_${tag}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c3 $tag rc=$rc"; exit $rc; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/c3_${tag}_$rep.log') if l.startswith('{')][-1]; print('$tag', d['value'], d['direct']['phase_share']['plan_frac'], d['direct']['all_ok'], d['bisection']['headers_per_s'])"
  done
done
