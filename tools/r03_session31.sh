#!/bin/bash
# Session 31: C2 PMC traffic passes on the round-3 final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s31
bash tools/pmc_pass.sh > gpurun_out/s31/pmc_c2.log 2>&1; rc=$?
tail -3 gpurun_out/s31/pmc_c2.log; exit $rc
