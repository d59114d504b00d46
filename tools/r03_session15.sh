#!/bin/bash
# Session 15: rare-column order A/B on C3 (then the relabel parity tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s15
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03l.txt || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_relabel.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/s15/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s15/pytest.log
exit $rc
