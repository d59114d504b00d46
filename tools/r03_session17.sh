#!/bin/bash
# Session 17 (round-3 final measurements): new tests, C2 / C3 bench lines with
# CPU baselines, rocprofv3 kernel stats, C3 PMC traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; O=gpurun_out/s17; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_relabel.py "tests/test_gpu_pm.py::test_pm_row_round_gradient" -x -q \
    --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== bench c2" && timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err && tail -c 300 $O/bench_c2.json && echo && \
echo "== bench c3" && timeout -k 10 500 python -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err && tail -c 300 $O/bench_c3.json && echo || exit 1
for cfg in "c2" "c3" "c2 --batch 8192"; do
  tag=$(echo $cfg | tr -d ' -'); args="--config $cfg"
  echo "== rocprofv3 $tag" && ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/$O/prof_$tag" -o run -- python3 "$R/bench.py" $args --no-cpu-baseline \
      > "$R/$O/prof_$tag.json" 2> "$R/$O/prof_$tag.err" ) || exit 1
done
echo "== pmc c3" && CONFIG=c3 STEPS=6 WARMUP=2 bash tools/pmc_pass.sh > $O/pmc_c3.log 2>&1 && tail -2 $O/pmc_c3.log
