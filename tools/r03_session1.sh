#!/bin/bash
# Round-3 first measurement session: bench arms (parity-order prices, C2
# batch sweep, C1 end to end), then the C2 gradient kernel's stamp timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/bench_arms.sh tools/arms/r03a.txt && \
echo "== c2 stamps" && timeout -k 10 300 python3 -u tools/c2_stamps.py > gpurun_out/arms/c2_stamps.txt 2>&1; \
cat gpurun_out/arms/c2_stamps.txt | tail -12
