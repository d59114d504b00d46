#!/bin/bash
# Round measurement session (one GPU box): GPU parity suite, smoke, C2 bench,
# rocprofv3 kernel-trace summaries of every config, PMC traffic passes for C2.
# Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/rp
if [ "${RP_TESTS:-1}" = 1 ]; then
echo "== pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/rp/pytest_gpu.log 2>&1 && tail -2 gpurun_out/rp/pytest_gpu.log && \
echo "== smoke" && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" && \
echo "== bench c2" && timeout -k 10 400 python -u bench.py > gpurun_out/rp/bench_c2.json 2> gpurun_out/rp/bench_c2.err && \
tail -c 400 gpurun_out/rp/bench_c2.json && echo || exit 1
fi

for cfg in ${RP_CONFIGS:-c1 c2 c3 c4 c5 c4s c2s}; do
  extra=""; [ $cfg = c4s ] && extra="--steps 12 --warmup 2"; [ $cfg = c2s ] && extra="--steps 50 --warmup 5"
  echo "== rocprofv3 $cfg" && ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/rp/prof_$cfg" -o run -- python3 "$R/bench.py" --config $cfg $extra --no-cpu-baseline \
      > "$R/gpurun_out/rp/prof_$cfg.json" 2> "$R/gpurun_out/rp/prof_$cfg.err" ) || exit 1
done && \
if [ "${RP_PMC:-1}" = 1 ]; then echo "== pmc" && bash tools/pmc_pass.sh > gpurun_out/rp/pmc_pass.log 2>&1; fi && \
echo "round profile done"
