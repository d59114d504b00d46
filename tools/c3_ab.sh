#!/bin/bash
# C3 bench A/B over env variants (C3_VARIANTS, ';'-separated), no tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c3ab
IFS=';' read -ra VARS <<< "${C3_VARIANTS:-DLR_MARGIN_HOT=1}"
k=0
for v in "${VARS[@]}"; do
  k=$((k+1))
  env $v timeout -k 10 300 python -u bench.py --config c3 --steps 6 --warmup 1 --no-cpu-baseline \
      > gpurun_out/c3ab/v$k.json 2> gpurun_out/c3ab/v$k.err || exit 1
  python - gpurun_out/c3ab/v$k.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"])
PY
done
