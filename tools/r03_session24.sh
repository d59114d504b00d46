#!/bin/bash
# Session 24: band pairs / long-phase pieces per lane 8 vs 4 (C3), parity of the variant first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s24
DLR_LIB=$(pwd)/dist-lr_amd/lib/libdistlr_amd_k2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bands.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/s24/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s24/pytest.log; [ $rc -eq 0 ] || exit $rc
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03r.txt
