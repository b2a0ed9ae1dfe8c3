#!/bin/bash
# Experiment: main-kernel time with the per-lane tables made L2-resident (wrong results; timing
# only) against the current build, plus the effective clock of each from one PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2f
mkdir -p $OUT
ROUNDS=2 STEPS=10 bash tools/ab.sh l2slab cur || exit $?
for v in l2slab cur; do
  if [ $v = cur ]; then lib=tendermint-fork_amd/lib/libtmed25519_hip.so; else lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so; fi
  TMED_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/pmc_$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-peak --no-c1 --no-keyset > $OUT/pmc_$v.log 2>&1 || exit $?
done
