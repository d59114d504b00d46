#!/bin/bash
# C3 iteration session: the C3-relevant GPU tests (bands, layouts, relabel,
# unit values), then the C3 bench with variants given in C3_VARIANTS
# (env assignments, ';'-separated), then a C3 kernel-trace profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c3i
timeout -k 10 500 python -u -m pytest tests/test_gpu_bands.py tests/test_gpu_layouts.py tests/test_gpu_relabel.py \
    tests/test_gpu_unit_values.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c3i/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/c3i/pytest.log; [ $rc = 0 ] || exit $rc
IFS=';' read -ra VARS <<< "${C3_VARIANTS:-DLR_MARGIN_HOT=1}"
k=0
for v in "${VARS[@]}"; do
  k=$((k+1))
  env $v timeout -k 10 300 python -u bench.py --config c3 --steps 6 --warmup 1 --no-cpu-baseline \
      > gpurun_out/c3i/v$k.json 2> gpurun_out/c3i/v$k.err || exit 1
  python - gpurun_out/c3i/v$k.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"])
PY
done
