#!/usr/bin/env python3
"""Parse the rocprofv3 PMC passes of tools/pmc_pass.sh into HBM traffic per
train step, calibrated on a known-byte stream.

FETCH_SIZE / WRITE_SIZE are kB derived from the L2's memory-side request
counters (MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE reads exactly half
the bytes of a wide coalesced streaming read).  The calibration pass runs
tools/kbench's mb_stream over cold 25 MiB windows (16-B loads per lane, known
bytes), so the read factor is measured here instead of assumed; it is applied
to the bench kernels' FETCH_SIZE.  Gathers (4-B loads, one line each) are not
calibrated by that stream; the raw counters are reported beside the
corrected figure.

    python tools/pmc_traffic.py gpurun_out/pmc  [--out profiles/traffic.json]
    python tools/pmc_traffic.py profiles/r02_pmc_c2      # the committed raw CSVs of profiles/traffic.json
    python tools/pmc_traffic.py profiles/r03_pmc_c3 --workload-key D16777216_nnz39_B-1 --layout classic \
        --steps 20 --out profiles/traffic_c3.json   # (bench --config c3 --steps 6 --warmup 2)
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def per_kernel(path: str, counter: str) -> dict[str, list[float]]:
    # rocprofv3's layout (<pass>/run_counter_collection.csv) or the flat copy
    # committed under profiles/ (<pass>.csv)
    if not os.path.exists(path):
        path = os.path.dirname(path) + ".csv"
    out: dict[str, list[float]] = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            out[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return out


def pick(d: dict[str, list[float]], key: str) -> list[float]:
    vals = []
    for name, v in d.items():
        if key in name:
            vals.extend(v)
    return vals


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--workload-key", default="D1000000_nnz50_B65536")
    ap.add_argument("--layout", default="lds", help="gradient layout the passes ran with (bench.py reports it)")
    ap.add_argument("--steps", type=int, default=0,
                    help="step-equivalents of the bench run (default: its margin dispatches; a band-pipelined "
                         "margin is dispatched once per band -- C3: warm-up + timed + stage-timing + breakdown steps)")
    args = ap.parse_args()
    d = args.pmc_dir
    # calibration: mb_stream reads 25 MiB and writes n4*4 bytes per launch
    win = 26214400
    n4 = win // 2 // 16
    cf = pick(per_kernel(os.path.join(d, "calib_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE"), "mb_stream")
    cw = pick(per_kernel(os.path.join(d, "calib_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE"), "mb_stream")
    read_factor = win / (statistics.median(cf) * 1024.0)
    write_factor = (n4 * 4) / (statistics.median(cw) * 1024.0)
    res = {"workload_key": args.workload_key, "layout": args.layout,
           "note": "L2-to-fabric bytes (FETCH_SIZE corrected by the calibration factor, WRITE_SIZE); Infinity-Cache "
                   "hits are counted, so gathered tables resident in MALL show here",
           "calibration": {"kernel": "kbench mb_stream, cold 25 MiB windows, 16-B loads per lane",
                           "read_bytes_true": win, "FETCH_SIZE_kB_median": statistics.median(cf),
                           "read_factor": round(read_factor, 4), "write_bytes_true": n4 * 4,
                           "WRITE_SIZE_kB_median": statistics.median(cw), "write_factor": round(write_factor, 4)},
           "kernels": {}}
    bf = per_kernel(os.path.join(d, "bench_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    bw = per_kernel(os.path.join(d, "bench_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    hits = per_kernel(os.path.join(d, "bench_TCC_HIT_sum_TCC_MISS_sum", "run_counter_collection.csv"), "TCC_HIT_sum")
    miss = per_kernel(os.path.join(d, "bench_TCC_HIT_sum_TCC_MISS_sum", "run_counter_collection.csv"), "TCC_MISS_sum")
    # Per train step: every dispatch of a stage's kernels summed, divided by
    # the number of steps (= margin dispatches: bench.py runs the margin and
    # the gradient stage equally often).  C2 has one kernel per stage; C3's
    # gradient is 12 band launches + long phases + combine + finalize.
    # Dense shards (C4): the fused pass is the margin role (it also forms the
    # gradient partials), the chunk combine + update the grad role.  Huge D
    # (C5): the dense L2 pass and the scatter are the update role.
    # Product margin (C2): pass 2 is the margin role, a separate pass 1
    # (k_pm_products) too; a fused pass 1 is inside k_grad_lds (grad role).
    # The product margin in the gradient's launch (k_grad_lds<F, true,
    # false, true, true>: pass 2 + gradient + update + next pass 1) is a step
    # of its own, like K6r.  A kernel counts in the first role that matches.
    # (round 5 added a sixth template argument, DB, round 6 removed it and
    # the NT argument: k_grad_lds<FILL, FUSED, PM, MG>; all spellings)
    mg = [", true, false, true, true>", ", true, false, true, true, ", "k_grad_lds<1, true, true, true>",
          "k_grad_lds<2, true, true, true>", "k_grad_lds<4, true, true, true>", "k_grad_lds<8, true, true, true>"]
    roles = [("margin", ["k_margin", "k_pm_margin", "k_pm_products", "k_dense_fused", "k_dense_margin", "k_flag_store"]),
             ("step", ["k_dense_ref<", *mg]),  # one launch: margin + gradient + update
             ("grad", ["k_grad", "k_long_", "k_band_finalize", "k_band_hot", "k_hot_chain", "k_dense_grad",
                       "k_dense_combine"]),
             ("update", ["k_dense_l2", "k_scatter", "k_merge_update", "k_sparse_merge"])]
    steps = args.steps or len([x for k in ["k_margin", "k_pm_margin", "k_dense_fused", "k_dense_margin", "k_dense_ref<",
                                           *mg] for x in pick(bf, k)]) or 1
    taken: set[str] = set()

    def take(d, keys):
        out = []
        for name, v in d.items():
            if name not in taken and any(k in name for k in keys):
                out.extend(v)
        return out

    total = 0.0
    for short, keys in roles:
        f, w, h, m = take(bf, keys), take(bw, keys), take(hits, keys), take(miss, keys)
        taken.update(n for d in (bf, bw, hits, miss) for n in d if any(k in n for k in keys))
        if not f:
            continue
        fk, wk = sum(f) / steps, (sum(w) / steps if w else 0.0)
        rd = fk * 1024.0 * read_factor
        wr = wk * 1024.0 * write_factor
        total += rd + wr
        res["kernels"][short] = {
            "dispatches": len(f), "dispatches_per_step": round(len(f) / steps, 2),
            "FETCH_SIZE_kB": round(fk, 1), "WRITE_SIZE_kB": round(wk, 1),
            "read_bytes": round(rd), "write_bytes": round(wr),
            "l2_hit_rate": round(sum(h) / (sum(h) + sum(m)), 4) if h and m else None,
        }
    res["hbm_bytes_per_step"] = round(total)
    js = json.dumps(res, indent=1)
    print(js)
    if args.out:
        with open(args.out, "w") as fo:
            fo.write(js + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
