#!/bin/bash
# Session 20: rare columns by (first band, second band, first occurrence) A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03o.txt
