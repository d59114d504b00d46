#!/bin/bash
# Session 16: C3 hot-tier width and band size with the rare-column order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03m.txt
