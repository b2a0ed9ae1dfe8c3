#!/bin/bash
# One GPU-box session: parity tests, bench, kernel-trace profile.  Every GPU step has its
# own time limit; a fault/abort/timeout (124/134/137/139) ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
nproc > $OUT/nproc.txt; lscpu > $OUT/lscpu.txt 2>&1; (which go || echo "no go") >> $OUT/nproc.txt 2>&1
STEPS="${*:-tests bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
      echo "tests rc=$rc" | tee -a $OUT/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc" | tee -a $OUT/smoke.log ;;
    bench)
      t0=$(date +%s); timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1; rc=$?; echo "bench wall $(( $(date +%s) - t0 )) s" >> $OUT/bench.log
      echo "bench rc=$rc" | tee -a $OUT/bench.log; tail -1 $OUT/bench.log ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline ${PROF_ARGS:-} > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; rc=$?
      cd $GRAFT_REPO_ROOT; echo "prof rc=$rc" | tee -a $OUT/prof.log ;;
    profc2)  # the C2 leg alone: every main-kernel launch is the full batch (its rocprof average = the roofline's)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/profc2 -o c2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-keyset --no-c1 --no-c4 --no-c3 --no-c5 --no-zip215 --steps 100 > $GRAFT_REPO_ROOT/$OUT/profc2.log 2>&1; rc=$?
      cd $GRAFT_REPO_ROOT; echo "profc2 rc=$rc" | tee -a $OUT/profc2.log ;;
    variants)
      rc=0
      IFS='|' read -ra VLIST <<< "${VARIANTS:-TMED_MAIN_WAVES=2|TMED_MAIN_WAVES=-2|TMED_MAIN_WAVES=3}"
      for cfg in "${VLIST[@]}"; do
        env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-peak --steps 5 > $OUT/variant.log 2>&1; rc=$?
        echo "$cfg rc=$rc $(tail -1 $OUT/variant.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)" | tee -a $OUT/variants.txt
        if fatal $rc; then break; fi
      done ;;
    merkle)
      timeout -k 10 300 python bench_merkle.py > $OUT/bench_merkle.log 2>&1; rc=$?
      echo "merkle rc=$rc"; grep '^{' $OUT/bench_merkle.log ;;
    keyset)
      timeout -k 10 300 python bench_keyset.py > $OUT/bench_keyset.log 2>&1; rc=$?
      echo "keyset rc=$rc"; grep '^{' $OUT/bench_keyset.log ;;
    commits)
      timeout -k 10 900 python bench_commits.py --config ${COMMITS_CFG:-c1,c3,c4} ${COMMITS_ARGS:-} > $OUT/bench_commits.log 2>&1; rc=$?
      echo "commits rc=$rc"; grep '^{' $OUT/bench_commits.log ;;
    probe)
      timeout -k 10 300 python tools/probe_valu.py > $OUT/probe_valu.json 2>$OUT/probe_valu.err; rc=$?
      echo "probe rc=$rc"; cat $OUT/probe_valu.json ;;
    counters)
      timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; rc=$? ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      rc=0
      PMC_SETS=${PMC_SETS:-"FETCH_SIZE|WRITE_SIZE|SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE|SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"}
      IFS='|' read -ra SETS <<< "$PMC_SETS"
      for ctr in "${SETS[@]}"; do
        tag=$(echo $ctr | tr ' ' '_')
        timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PMC_ARGS---no-peak} --c1-reps 50 --no-c4 --no-c5 --no-zip215 > $GRAFT_REPO_ROOT/$OUT/pmc_$tag.log 2>&1; rc=$?
        echo "pmc $ctr rc=$rc" | tee -a $GRAFT_REPO_ROOT/$OUT/pmc.log
        if fatal $rc; then break; fi
      done
      cd $GRAFT_REPO_ROOT ;;
    *) echo "unknown step $s"; rc=0 ;;
  esac
  if fatal $rc; then echo "fatal rc=$rc in $s; stopping"; exit $rc; fi
done
exit 0
