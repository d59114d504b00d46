#!/bin/bash
# pipelined chain reads (c4x), clamped C2 windows: parity subsets, stamps, bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_dense.py tests/test_gpu_fullsize.py \
    -k "not c3_eight and not c3_full_size and not fused" -q --timeout 400 --timeout-method thread \
    > gpurun_out/s4/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" gpurun_out/s4/pytest.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/c2_stamps.py > gpurun_out/s4/stamps.txt 2>&1 && grep -v amdgpu.ids gpurun_out/s4/stamps.txt && \
bash tools/bench_arms.sh tools/arms/r03c.txt
