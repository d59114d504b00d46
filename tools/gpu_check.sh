#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile.  Every GPU step
# has its own time limit and the steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
echo "== smoke" && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" && \
echo "== bench" && timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cat gpurun_out/bench.json && \
echo "== rocprofv3 kernel trace" && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" \
    -o bench --output-format csv -- python3 "$R/bench.py" --steps 500 --warmup 20 --no-cpu-baseline \
    > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" && echo "profile done"
