#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 --pmc runs: for every kernel (name
shortened to its template head), the median over its dispatches of each
counter (a dispatch's rows summed first), plus the median kernel duration.

  python tools/pmc_summary.py gpurun_out/diag_c2/p1 gpurun_out/diag_c2/p2 ...
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import statistics
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("dlr::", "")
    name = name.split("(")[0]
    return name if len(name) < 90 else name[:87] + "..."


def load(d: str):
    out = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k, disp, c = short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"]
                out[k][c][disp] = out[k][c].get(disp, 0.0) + float(r["Counter_Value"])
                dur[k][disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return out, dur


def main():
    merged = collections.defaultdict(dict)
    durs = collections.defaultdict(list)
    for d in sys.argv[1:]:
        out, dur = load(d)
        for k, cs in out.items():
            for c, per in cs.items():
                merged[k][c] = statistics.median(per.values())
            durs[k].extend(dur[k].values())
    for k in sorted(merged, key=lambda k: -statistics.median(durs[k])):
        if k.startswith("__amd"):
            continue
        print(f"{k}  (median {statistics.median(durs[k]):.2f} us under counters, {len(durs[k])} dispatches)")
        for c in sorted(merged[k]):
            print(f"  {c:32s} {merged[k][c]:14.4g}")


if __name__ == "__main__":
    main()
