#!/usr/bin/env python3
"""Where the C3 margin's gathers land: the histogram of the entries' column
ranks after the engine's frequency relabeling (rank 0 = the most frequent
column), and how many 8 MB rank slices a row's cold entries touch.  Host
only (numpy over the seeded generator); DESIGN.md §5 quotes its output.

    python tools/c3_ranks.py [rows]          # default: C3's 12.5M rows per GPU
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dist-lr_amd"))
import distlr_amd as dlr  # noqa: E402


def main() -> None:
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
    D = 1 << 24
    ds = dlr.Dataset.generate_hashed(rows, D, 39, seed=10, stream=1)
    rp, col, _val, lab = ds.csr()
    cnt = np.bincount(col, minlength=D)
    order = np.argsort(-cnt, kind="stable")
    rank = np.empty(D, np.int32)
    rank[order] = np.arange(D, dtype=np.int32)
    r = rank[col]
    del col
    edges = [0, 1 << 14, 1 << 18, 1 << 20, 1 << 21, 1 << 22, 1 << 23, 1 << 24]
    h = np.histogram(r, bins=edges)[0]
    print(f"C3 shard: {rows} rows, {len(r)} entries, {int((cnt > 0).sum())} distinct columns")
    for a, b, n in zip(edges, edges[1:], h):
        print(f"  ranks [{a:>9}, {b:>9}): {n / len(r):.3f} of entries")
    cold = r >= (1 << 14)
    row_of = np.repeat(np.arange(len(lab), dtype=np.int64), np.diff(rp))
    key = np.unique(row_of[cold] * 8 + (r[cold] >> 21))
    per = np.bincount(key // 8, minlength=len(lab))
    print(f"  cold entries per row {cold.sum() / len(lab):.2f}; distinct 8 MB rank slices they touch per row: "
          f"{per.mean():.2f} of 8")


if __name__ == "__main__":
    main()
