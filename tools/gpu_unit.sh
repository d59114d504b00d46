#!/bin/bash
# Unit-valued shards: full GPU parity suite, then C3 / C5 bench lines with
# the UNIT kernels (default) and with the value arrays kept (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/unit
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/unit/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/unit/pytest.log; [ $rc = 0 ] || exit $rc
for cfg in c3 c5; do
  for u in 1 0; do
    DLR_UNIT_VALUES=$u timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline \
        > gpurun_out/unit/b_${cfg}_u$u.json 2> gpurun_out/unit/b_${cfg}_u$u.err || exit 1
  done
done
python - <<'PY'
import json
for cfg in ["c3", "c5"]:
    for u in ["1", "0"]:
        d = json.loads(open(f"gpurun_out/unit/b_{cfg}_u{u}.json").read().strip().splitlines()[-1])
        r = d["roofline"]
        print(cfg, "unit" if u == "1" else "valued", d["value"], d["ms_per_step"], r["kernel_avg_us"], r["frac"])
PY
