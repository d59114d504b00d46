#!/bin/bash
# long-run band variant (c3x): C3 parity subsets, then c3x / c3 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s6
timeout -k 10 900 python -u -m pytest tests/test_gpu_bands.py tests/test_gpu_fullsize.py tests/test_gpu_c3_full.py \
    -k "not dense" -q --timeout 600 --timeout-method thread > gpurun_out/s6/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" gpurun_out/s6/pytest.log | tail -15
[ $rc -eq 0 ] || exit $rc
bash tools/bench_arms.sh tools/arms/r03e.txt
