#!/bin/bash
# Session 34 (round-3 final library, rebuilt after the reverted A/B): the whole GPU suite as the driver runs it,
# smoke, the default bench line, the B = 8,192 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s34
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --durations=12 --timeout 600 --timeout-method thread \
    > gpurun_out/s34/pytest.log 2>&1; rc=$?
tail -18 gpurun_out/s34/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s34/bench.json 2> gpurun_out/s34/bench.err && \
tail -c 300 gpurun_out/s34/bench.json && echo && \
timeout -k 10 300 python -u bench.py --batch 8192 --steps 1000 --warmup 50 --no-cpu-baseline > gpurun_out/s34/bench_b8192.json 2> gpurun_out/s34/bench_b8192.err && \
python3 -c "import json;d=json.loads(open('gpurun_out/s34/bench_b8192.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['config']['gradient_layout'])" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s34/prof -o c2 -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s34/prof.log 2>&1
