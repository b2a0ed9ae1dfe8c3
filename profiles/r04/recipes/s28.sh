#!/bin/bash
# Round-4 session 28: the keyed latency kernel finishing a batch of <= 256 signatures in its last
# block (no finish kernel): -m gpu suite, then C1 alternating with the previous build
# (lib/ab/libtmed_latsplit.so), three runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s28
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for L in tendermint-fork_amd/lib/ab/libtmed_latsplit.so tendermint-fork_amd/lib/libtmed25519_hip.so; do
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
