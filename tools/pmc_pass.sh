#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, as the gfx950 slot limits
# require) over the bench workload and a known-byte calibration stream.
# Output: gpurun_out/pmc/<pass>/...  (parsed by tools/pmc_traffic.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
PD=gpurun_out/pmc${CONFIG:+_$CONFIG}
mkdir -p $PD
STEPS=${STEPS:-40}
cd /tmp
for pass in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | tr ' ' '_')
  echo "== pass $tag (calibration)"
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$R/$PD/calib_$tag" -o run -- \
      "$R/tools/kbench/kbench" 65536 1000000 50 40 calib > "$R/$PD/calib_$tag.log" 2>&1 || exit 1
  echo "== pass $tag (bench)"
  timeout -s KILL 400 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$R/$PD/bench_$tag" -o run -- \
      python3 "$R/bench.py" ${CONFIG:+--config $CONFIG} --steps $STEPS --warmup ${WARMUP:-5} --no-cpu-baseline \
      ${NO_STAGES:+--no-stage-pass} > "$R/$PD/bench_$tag.json" \
      2> "$R/$PD/bench_$tag.err" || exit 1
done
echo "pmc passes done"
