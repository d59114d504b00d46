#!/bin/bash
# Session 22: product chunks without padding (pass-1 tail groups stored slot by slot).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s22
timeout -k 10 400 python -u -m pytest tests/test_gpu_pm.py tests/test_gpu_layouts.py tests/test_gpu_multirank.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/s22/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s22/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
ARM_TIMEOUT=300 bash tools/bench_arms.sh tools/arms/r03q.txt
