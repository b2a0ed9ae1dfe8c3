#!/bin/bash
# Round-5 closing session: full -m gpu suite, smoke, bench.py (the driver's default command), a
# rocprofv3 kernel-trace summary of the same bench and of its C2 leg alone, PMC passes (the VALU peak probe included, for
# the clock comparison).  Steps and limits: tools/gpu_check.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PMC_ARGS="" bash tools/gpu_check.sh ${*:-tests smoke bench prof profc2 pmc}
