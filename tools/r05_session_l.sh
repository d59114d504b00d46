#!/bin/bash
# round 5: C4 stamps with and without the paced start; C3 reference-order PMC
# traffic (whole steps only) and its rocprof kernel summary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05l
mkdir -p $O
DLR_DENSE_REF_PACE=0 timeout -k 10 300 python -u tools/c4_stamps.py > $O/st_c4_p0.txt 2>&1 || exit 1
DLR_DENSE_REF_PACE=170 timeout -k 10 300 python -u tools/c4_stamps.py > $O/st_c4_p170.txt 2>&1 || exit 1
CONFIG=c3 STEPS=6 WARMUP=2 NO_STAGES=1 timeout -k 10 1000 bash tools/pmc_pass.sh || exit 1
echo done
