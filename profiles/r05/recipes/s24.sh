#!/bin/bash
# Round-5 session 24: rocprofv3 kernel-trace summary of bench.py's C2 leg alone (every launch of
# verify_main_hs_kernel<26> is then the full 2^20 batch, so its rocprof average is directly the
# roofline's kernel_avg_ms), with the bench line of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s24
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-keyset --no-c1 --no-c4 --no-c3 --no-c5 --no-zip215 --steps 100 > $GRAFT_REPO_ROOT/$O/bench_c2only.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -c 300 $GRAFT_REPO_ROOT/$O/bench_c2only.log
exit $rc
