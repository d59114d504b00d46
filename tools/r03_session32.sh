#!/bin/bash
# Session 32: rocprofv3 kernel stats of the C3 line at the 2,048 threshold.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/s32; export TMPDIR=/tmp
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/s32/prof_c3" -o run -- \
    python3 "$R/bench.py" --config c3 --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/s32/bench_c3.json" 2> "$R/gpurun_out/s32/bench_c3.err"
