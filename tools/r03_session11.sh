#!/bin/bash
# Session 11: per-workgroup timelines of k_grad_rt and k_grad_lds (stamps build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s11
timeout -k 10 200 python -u tools/c2_stamps.py > gpurun_out/s11/rt.txt 2>&1 && cat gpurun_out/s11/rt.txt && \
timeout -k 10 200 python -u tools/c2_stamps.py --lds > gpurun_out/s11/lds.txt 2>&1 && cat gpurun_out/s11/lds.txt
