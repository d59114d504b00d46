#!/bin/bash
# 256-row chain slots (c4x), the exchange / next-margin overlap (loopback + 1-rank RCCL)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s5
timeout -k 10 700 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_dense.py tests/test_gpu_fullsize.py \
    tests/test_gpu_multirank.py -k "not c3_eight and not c3_full_size and not fused" -q --timeout 400 \
    --timeout-method thread > gpurun_out/s5/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" gpurun_out/s5/pytest.log | tail -15
[ $rc -eq 0 ] || exit $rc
bash tools/bench_arms.sh tools/arms/r03d.txt
