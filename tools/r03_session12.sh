#!/bin/bash
# Session 12: RT with every round's entries issued up front (A/B + timeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s12
DLR_LIB=$(pwd)/dist-lr_amd/lib/libdistlr_amd_rtup.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pm.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/s12/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s12/pytest.log
[ $rc -eq 0 ] || exit $rc
DLR_LIB=$(pwd)/dist-lr_amd/lib/libdistlr_amd_stamps_rtup.so timeout -k 10 200 python -u tools/c2_stamps.py > gpurun_out/s12/rtup.txt 2>&1 && cat gpurun_out/s12/rtup.txt && \
ARM_TIMEOUT=300 bash tools/bench_arms.sh tools/arms/r03i.txt
