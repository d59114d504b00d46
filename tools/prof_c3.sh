#!/bin/bash
# C3 kernel-trace profile (rocprofv3 --stats), per-kernel averages printed.
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/pc3
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pc3" -o run -- python3 "$R/bench.py" --config c3 --steps 6 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pc3/b.json" 2> "$R/gpurun_out/pc3/b.err" || exit 1
python3 - "$R/gpurun_out/pc3/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s %5s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000))
PY
