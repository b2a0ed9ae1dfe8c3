#!/bin/bash
# Round-5 session 4: C3 host phases traced; C3 + C4 with the reworked compiled marshal; one PMC pass
# (GRBM_GUI_ACTIVE: effective clock of the main kernel beside the VALU peak probe's, same run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s4
mkdir -p $O
TMED_TRACE=1 timeout -k 10 300 python bench_commits.py --config c3 --runs 3 > $O/c3_trace.log 2>&1; rc=$?
echo "c3 trace rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench_commits.py --config c3,c4 --runs 5 --blocks 12500 > $O/commits.log 2>&1; rc=$?
echo "commits rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/$O/pmc_clock -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-keyset --no-c1 --no-c3 --no-c4 --no-c5 --no-zip215 > $R/$O/pmc_clock.log 2>&1; rc=$?
echo "pmc rc=$rc"
cd $R && python3 tools/pmc_summary.py $O/pmc_clock.json $O/pmc_clock > /dev/null 2>&1
exit $rc
