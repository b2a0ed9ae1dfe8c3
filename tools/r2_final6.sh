#!/bin/bash
# Round-2 end-of-session measurement set (final6): GPU parity suite, smoke, the default bench line (every leg), a
# rocprofv3 kernel-trace profile of the bench and the PMC passes behind roofline.traffic /
# the VALU issue split / the effective clock.  Every GPU step has its own time limit; the
# session stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final6
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
grep '^{' $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-keyset > $OUT/prof.log 2>&1 || exit $?
echo "prof ok"
n=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc$n -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-peak --no-c1 --no-keyset > $OUT/pmc$n.log 2>&1 || exit $?
  echo "pmc $n ok"
done
cd $R
TMED_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --sigs 262144 --steps 10 --no-cpu-baseline --no-c1 --no-keyset > $OUT/bench_2ranks.log 2>&1 || exit $?
grep '^{' $OUT/bench_2ranks.log | cut -c1-200
timeout -k 10 900 python -u bench_commits.py --config c3,c4 > $OUT/bench_commits.jsonl 2> $OUT/bench_commits.err || exit $?
echo "commits ok"
