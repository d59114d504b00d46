#!/bin/bash
# Session 33: per-band long-column phases (DLR_LONG_PERBAND=1): bitwise vs
# the sequential order, then A/B on the C3 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s33
timeout -k 10 300 python -u -m pytest tests/test_gpu_bands.py -x -q -k "per_band or pipeline_bitwise" --timeout 200 --timeout-method thread \\
    > gpurun_out/s33/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/s33/pytest.log; [ $rc -eq 0 ] || exit $rc
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03x.txt
