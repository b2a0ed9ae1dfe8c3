#!/bin/bash
# Round 5 s31: occupancy of the full-size C2 launches (bench.py's C2 leg alone): SQ_WAVE_CYCLES,
# SQ_BUSY_CYCLES, SQ_WAVES, GRBM_GUI_ACTIVE per dispatch, to size the main kernel's tail.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/s31
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
  --output-format csv -d $PWD/gpurun_out/s31/pmc -o run -- python3 $PWD/bench.py --steps 10 --warmup 2 --no-cpu-baseline \
  --no-keyset --no-c1 --no-c4 --no-c3 --no-c5 --no-zip215 > gpurun_out/s31/pmc.log 2>&1
echo "pmc rc=$?"
