#!/bin/bash
# Diagnostic PMC passes (one counter group per rocprofv3 run) over one bench
# config, to see what bounds its kernels: instruction mix and wait states
# (SQ), L2 hits / misses / fabric requests (TCC), L1 / texture units.
#   CONFIG=c3 bash tools/pmc_diag.sh   -> gpurun_out/diag_<config>/<pass>/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
CONFIG=${CONFIG:-c2}
PD=gpurun_out/diag_$CONFIG
mkdir -p $PD
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/$PD/avail.txt" 2>&1 || true
IFS=';' read -ra PASSES <<< "${PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES;SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum;TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum}"
k=0
for pass in "${PASSES[@]}"; do
  k=$((k+1))
  echo "== pass $k: $pass"
  timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$R/$PD/p$k" -o run -- \
      python3 "$R/bench.py" --config $CONFIG --steps ${STEPS:-3} --warmup ${WARMUP:-1} --no-cpu-baseline \
      > "$R/$PD/p$k.json" 2> "$R/$PD/p$k.err" || { echo "pass $k failed"; tail -5 "$R/$PD/p$k.err"; }
done
echo "diag passes done"
