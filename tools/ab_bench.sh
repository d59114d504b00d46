#!/bin/bash
# A/B of environment knobs on the bench workload, one box: each arm under
# rocprofv3 --kernel-trace --stats; prints per-kernel average durations.
#   ARMS="DLR_GRAD_NT=1 DLR_GRAD_NT=0" bash tools/ab_bench.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/ab
cd /tmp
i=0
for arm in ${ARMS:-base}; do
  i=$((i+1))
  env $( [ "$arm" = base ] || echo $arm ) true
  ( [ "$arm" = base ] || export $arm
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ab/arm$i" -o run -- \
      python3 "$R/bench.py" --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline > "$R/gpurun_out/ab/arm$i.json" 2> "$R/gpurun_out/ab/arm$i.err" ) || exit 1
  echo "== arm $i: $arm  value=$(python3 -c "import json;print(json.loads(open('$R/gpurun_out/ab/arm$i.json').read().strip().splitlines()[-1])['value'])")"
  python3 - "$R/gpurun_out/ab/arm$i/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 100:
        print("   %-60s %9.2f us" % (r["Name"][:60], float(r["AverageNs"]) / 1000))
PY
done
