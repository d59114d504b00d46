#!/bin/bash
# Session 26: c2s / c1 without the profiler (regression check).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03s.txt
