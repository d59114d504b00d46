#!/bin/bash
# pipelined long-run band windows (c3x): C3 parity subsets, then the c3x line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s7
timeout -k 10 900 python -u -m pytest tests/test_gpu_bands.py tests/test_gpu_fullsize.py tests/test_gpu_layouts.py \
    -k "not dense and not default" -q --timeout 600 --timeout-method thread > gpurun_out/s7/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" gpurun_out/s7/pytest.log | tail -15
[ $rc -eq 0 ] || exit $rc
bash tools/bench_arms.sh tools/arms/r03f.txt
