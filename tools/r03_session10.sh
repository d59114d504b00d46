#!/bin/bash
# Session 10: RT without scratch + fixed-stride pass-2 regions: parity, C2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s10
timeout -k 10 300 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_layouts.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/s10/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/s10/pytest.log
[ $rc -eq 0 ] || exit $rc
ARM_TIMEOUT=300 bash tools/bench_arms.sh tools/arms/r03h.txt
