#!/bin/bash
# Several bench.py lines on one GPU box, each with its own environment and
# arguments; every arm has its own time limit and the arms are chained (the
# first failure ends the call).
#   bash tools/bench_arms.sh tools/arms/r03a.txt   (lines: name|ENV=V ...|bench args)
# -> gpurun_out/arms/<name>.json (+ .err); prints each line's value / frac.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/arms
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  echo "== $name: env [$envs] args [$args]"
  env $envs timeout -k 10 "${ARM_TIMEOUT:-420}" python3 -u "$R/bench.py" $args ${ARM_EXTRA---no-cpu-baseline} < /dev/null \
      > "gpurun_out/arms/$name.json" 2> "gpurun_out/arms/$name.err" || { tail -5 "gpurun_out/arms/$name.err"; exit 1; }
  python3 - "gpurun_out/arms/$name.json" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]
print("   value %.4g samples/s  ms/step %.5f  frac %s  kernels %s  layout %s  margin %s" % (
    j["value"], j["ms_per_step"], r["frac"], r["kernel_avg_us"], j["config"]["gradient_layout"],
    j["config"]["margin"]))
PY
done < "$1"
echo "arms done"
