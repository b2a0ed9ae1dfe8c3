#!/bin/bash
# C4 device-time attribution: a kernel + memory-copy trace of the blocksync leg (one GPU's
# shard shape: 10k validators, 128-block batches), plus the seam's own TMED_TRACE timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out/c4t
cd /tmp && export TMPDIR=/tmp
TMED_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/c4t/prof -o run --output-format csv -- python3 $R/bench_commits.py --config c4 --blocks 2000 --no-cpu > $R/gpurun_out/c4t/c4.log 2>&1
echo "c4 trace rc=$?"
