#!/bin/bash
# Kernel-trace profile of one bench config (rocprofv3 --kernel-trace --stats):
#   CFG=c4 bash tools/prof_cfg.sh  -> gpurun_out/pcfg_<cfg>/run_kernel_{trace,stats}.csv
# then prints per-kernel averages and the median gap between consecutive kernels
# of the timed loop.
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; CFG=${CFG:-c4}; O=$R/gpurun_out/pcfg_$CFG; mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- \
    python3 "$R/bench.py" --config $CFG ${BENCH_ARGS:-} --no-cpu-baseline > "$O/b.json" 2> "$O/b.err" || exit 1
python3 - "$O" <<'PY'
import csv, statistics, sys
o = sys.argv[1]
for r in csv.DictReader(open(o + "/run_kernel_stats.csv")):
    print("%-70s %5s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000))
rows = sorted(csv.DictReader(open(o + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000 for a, b in zip(rows, rows[1:])]
print("kernels %d, median gap %.2f us, mean gap (gaps < 100 us) %.2f us" %
      (len(rows), statistics.median(gaps), statistics.mean([g for g in gaps if g < 100])))
PY
