#!/bin/bash
# Session 21: k_grad_lds with 8 waves x 8 column groups (A/B) -- parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s21
DLR_GRAD_RT=0 DLR_LIB=$(pwd)/dist-lr_amd/lib/libdistlr_amd_w8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pm.py -x -q -k "not row_round" \
    --timeout 120 --timeout-method thread > gpurun_out/s21/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s21/pytest.log; [ $rc -eq 0 ] || exit $rc
ARM_TIMEOUT=300 bash tools/bench_arms.sh tools/arms/r03p.txt
