#!/bin/bash
# Session 14: first-occurrence order of the rare columns (C3 margin): parity, A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s14
timeout -k 10 500 python -u -m pytest tests/test_gpu_relabel.py tests/test_gpu_c3_full.py tests/test_gpu_bands.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/s14/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s14/pytest.log
[ $rc -eq 0 ] || exit $rc
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03k.txt
