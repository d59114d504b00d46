#!/bin/bash
# Iteration session: GPU parity tests (both gradient layouts), then bench
# with the default (LDS) and the classic gradient kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/it_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/it_pytest.log; [ $rc = 0 ] || exit $rc
DLR_GRAD_KERNEL=classic timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/it_pytest_classic.log 2>&1; rc=$?; tail -2 gpurun_out/it_pytest_classic.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err || exit 1
DLR_GRAD_KERNEL=classic timeout -k 10 300 python -u bench.py --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/it_bench_classic.json 2>> gpurun_out/it_bench.err || exit 1
python - <<'PY'
import json
for f in ["gpurun_out/it_bench.json", "gpurun_out/it_bench_classic.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"])
PY
