#!/bin/bash
# Session 19 (round-3 close): the whole GPU suite as the driver runs it
# (-x), smoke, the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s19
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 600 --timeout-method thread \
    > gpurun_out/s19/pytest.log 2>&1; rc=$?
tail -22 gpurun_out/s19/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s19/bench.json 2> gpurun_out/s19/bench.err && \
tail -c 600 gpurun_out/s19/bench.json
