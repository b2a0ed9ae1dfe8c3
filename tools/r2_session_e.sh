#!/bin/bash
# A/B only (no tests): VARS="a b c" ROUNDS=n
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROUNDS=${ROUNDS:-2} bash tools/ab.sh ${VARS:-cols cur}
