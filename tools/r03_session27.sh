#!/bin/bash
# Session 27: C3 long-column threshold with the rare-column order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03t.txt
