#!/bin/bash
# End-of-round measurement: GPU parity suite, smoke, the default bench line (every leg), a
# rocprofv3 kernel-trace profile, and a 2-rank rehearsal of bench.py's own rank spawning (gloo
# on the one GPU of this box; the driver's multi-GPU runs use RCCL).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | cut -c1-200
TMED_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --sigs 262144 --steps 10 --no-cpu-baseline --no-c1 --no-keyset > $OUT/bench_2ranks.log 2>&1 || exit $?
grep '^{' $OUT/bench_2ranks.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-keyset > $OUT/prof.log 2>&1 || exit $?
echo "prof ok"
