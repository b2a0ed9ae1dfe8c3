#!/bin/bash
# Round-4 final session: full -m gpu suite, smoke, bench.py (the driver's default command), a
# rocprofv3 kernel-trace summary of the same bench, PMC passes for the roofline traffic, probes.
# Steps and limits: tools/gpu_check.sh (a fault/abort/timeout ends the session there).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_check.sh ${*:-tests smoke bench prof pmc}
