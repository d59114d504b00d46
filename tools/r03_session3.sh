#!/bin/bash
# C2 gradient prologue rework + the reference-order dense gradient (chain):
# parity tests first, then stamps, then bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s3
timeout -k 10 900 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_layouts.py tests/test_gpu_dense.py \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "not c3_eight and not c3_full_size" -q --timeout 600 \
    --timeout-method thread -s > gpurun_out/s3/pytest.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed|fused dense" gpurun_out/s3/pytest.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 200 python3 -u tools/c2_stamps.py > gpurun_out/s3/stamps.txt 2>&1 && grep -v amdgpu.ids gpurun_out/s3/stamps.txt && \
bash tools/bench_arms.sh tools/arms/r03b.txt
