#!/bin/bash
# Session 25: round-3 lines of the configs whose kernels did not change (no
# regression check): c1, c4, c5, c2s bench lines + rocprofv3 summaries.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; O=gpurun_out/s25; mkdir -p $O
for cfg in c1 c4 c5 c2s; do
  extra=""; [ $cfg = c2s ] && extra="--steps 50 --warmup 5"
  echo "== $cfg" && ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$O/prof_$cfg" -o run -- python3 "$R/bench.py" --config $cfg $extra --no-cpu-baseline \
      > "$R/$O/prof_$cfg.json" 2> "$R/$O/prof_$cfg.err" ) || exit 1
  python3 -c "import json;d=json.loads(open('$O/prof_$cfg.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
done
