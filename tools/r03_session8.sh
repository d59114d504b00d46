#!/bin/bash
# Session 8 (re-entry): the whole GPU suite with per-test durations, then smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s8
timeout -k 10 1080 python -u -m pytest tests -m gpu -q --durations=40 --timeout 600 --timeout-method thread \
    > gpurun_out/s8/pytest.log 2>&1; rc=$?
tail -60 gpurun_out/s8/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()"
