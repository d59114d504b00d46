#!/bin/bash
# Session 29: C3 piece size, band rows and rare-column bound at the 2,048 threshold.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03v.txt
