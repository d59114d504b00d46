#!/bin/bash
# Session 13: RT with fixed-stride rounds, entries up front: parity, timeline, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s13
timeout -k 10 300 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_layouts.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/s13/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s13/pytest.log
[ $rc -eq 0 ] || exit $rc
DLR_GRAD_RT=1 timeout -k 10 200 python -u tools/c2_stamps.py > gpurun_out/s13/rt.txt 2>&1 && cat gpurun_out/s13/rt.txt && \
ARM_TIMEOUT=300 bash tools/bench_arms.sh tools/arms/r03j.txt
