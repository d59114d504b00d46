#!/bin/bash
# Session 28: band-mode long-column threshold 2,048 -- the C3 tolerance and
# determinism tests, then the C3 line with the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s28
timeout -k 10 700 python -u -m pytest tests/test_gpu_c3_full.py tests/test_gpu_bands.py tests/test_gpu_fullsize.py \
    tests/test_gpu_multirank.py tests/test_gpu_relabel.py -x -q -k "not dense and not c4" --timeout 400 --timeout-method thread \
    > gpurun_out/s28/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/s28/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config c3 > gpurun_out/s28/bench_c3.json 2> gpurun_out/s28/bench_c3.err && \
python3 -c "import json;d=json.loads(open('gpurun_out/s28/bench_c3.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_us'])"
