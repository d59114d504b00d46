#!/bin/bash
# Session 9: row-round gradient (RT) parity + C2 A/B; then the unit-values
# fault of session 8 isolated (kernels serialized, verbose order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s9
timeout -k 10 400 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_layouts.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/s9/pytest_rt.log 2>&1; rc=$?
tail -5 gpurun_out/s9/pytest_rt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
ARM_TIMEOUT=300 bash tools/bench_arms.sh tools/arms/r03g.txt || exit 1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_stream_sparse.py tests/test_gpu_unit_values.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/s9/pytest_unit.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/s9/pytest_unit.log | tail -30
exit $rc
