#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace) of the default build and of a prep experiment.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=$GRAFT_REPO_ROOT/gpurun_out/r2i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in cur ${VARIANTS:-}; do
  if [ "$v" = cur ]; then lib=$GRAFT_REPO_ROOT/tendermint-fork_amd/lib/libtmed25519_hip.so; else lib=$GRAFT_REPO_ROOT/tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so; fi
  TMED_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-keyset ${BENCH_ARGS:-} > $OUT/$v.log 2>&1 || exit $?
  echo "== $v"; tail -1 $OUT/$v.log | cut -c1-400
  f=$(find $OUT/$v -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -14
done
