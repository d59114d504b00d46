#!/bin/bash
# Row-band iteration session: band parity tests (+ the layout suite), then
# the C3 bench with bands off / 2^18 / 2^19 / 2^20 rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/band
timeout -k 10 500 python -u -m pytest tests/test_gpu_bands.py tests/test_gpu_layouts.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/band/pytest.log 2>&1; rc=$?; tail -4 gpurun_out/band/pytest.log; [ $rc = 0 ] || exit $rc
for br in ${BAND_SWEEP:-0 262144 524288 1048576}; do
  DLR_BAND_ROWS=$br timeout -k 10 300 python -u bench.py --config c3 --steps 6 --warmup 1 --no-cpu-baseline \
      > gpurun_out/band/c3_$br.json 2> gpurun_out/band/c3_$br.err || exit 1
  python - gpurun_out/band/c3_$br.json $br <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"]["gradient_layout"], d["roofline"]["kernel_avg_us"])
PY
done
