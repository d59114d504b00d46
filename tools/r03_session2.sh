#!/bin/bash
# C2 gradient-kernel timeline: stamps build and its ablation / variant builds,
# then the new GPU tests (full-size reference orders, W = 8 loopback, abort).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s2
for v in "" _abl1 _abl2 _abl4 _abl8 _abl16; do
  DLR_LIB=$PWD/dist-lr_amd/lib/libdistlr_amd_stamps$v.so timeout -k 10 200 python3 -u tools/c2_stamps.py \
      > gpurun_out/s2/stamps$v.txt 2>&1 || { tail -5 gpurun_out/s2/stamps$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/s2/stamps$v.txt
done
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -k "fullsize or failed_rank or c3_eight or fused_dense_c4 or reference_order" \
    -v --timeout 600 --timeout-method thread -s > gpurun_out/s2/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/s2/pytest.log | tail -20
exit $rc
