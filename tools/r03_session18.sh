#!/bin/bash
# Session 18: slab-free long phases (C3): bitwise vs the slab kernel, A/B;
# the C3 PMC traffic passes (kbench now travels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s18
timeout -k 10 400 python -u -m pytest tests/test_gpu_bands.py tests/test_gpu_c3_full.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/s18/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/s18/pytest.log
[ $rc -eq 0 ] || exit $rc
ARM_TIMEOUT=400 bash tools/bench_arms.sh tools/arms/r03n.txt || exit 1
echo "== pmc c3" && CONFIG=c3 STEPS=6 WARMUP=2 bash tools/pmc_pass.sh > gpurun_out/s18/pmc_c3.log 2>&1; tail -3 gpurun_out/s18/pmc_c3.log
