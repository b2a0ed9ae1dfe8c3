#!/bin/bash
# Round-4 session 20: C1 latency with column sums + separate carry pass in the kernels
# (TMED_FE_FUSED=0: ten independent column chains, then two interleaved carry chains) against
# the fused carry (one serial chain through all columns), alternating, three runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s20
mkdir -p $O
for rep in 1 2 3; do
  for L in tendermint-fork_amd/lib/libtmed25519_hip.so tendermint-fork_amd/lib/ab/libtmed_unfused.so; do
    tag=$(basename $L .so)
    TMED_LIB=$PWD/$L timeout -k 10 200 python bench_commits.py --config c1 > $O/c1_${tag}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c1 $tag rc=$rc"; exit $rc; }
    python3 - "$O/c1_${tag}_$rep.log" "$tag" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
p = d.get('paths', d)
print(sys.argv[2], json.dumps({k: (v.get('p50_ms') if isinstance(v, dict) else v) for k, v in p.items() if isinstance(v, dict)}))
PY
  done
done
