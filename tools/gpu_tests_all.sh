#!/bin/bash
# All GPU tests without stopping at the first failure (diagnosis runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_gpu_all.log
exit $rc
