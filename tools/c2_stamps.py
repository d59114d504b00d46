#!/usr/bin/env python3
"""Per-workgroup timeline of the C2 gradient kernel (k_grad_rt, or
k_grad_lds with --lds; both with the fused pass 1) from s_memrealtime stamps
(100 MHz), on the bench's C2 shard
shape.  Loads the DLR_STAMPS build of the library (make -C dist-lr_amd
stamps) through DLR_LIB.  Development tool, never part of the product.

  python tools/c2_stamps.py [--rows N] [--steps K] [--reps R]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DLR_LIB", os.path.join(ROOT, "dist-lr_amd", "lib", "libdistlr_amd_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "dist-lr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (one HIP runtime: torch's)

import distlr_amd as dlr  # noqa: E402

SLOTS = {11: "mg start", 12: "mg p2 pub", 14: "mg p2 pub w3", 13: "mg ph0 ok", 0: "start", 8: "win0+fill0 out", 9: "w0 drained", 10: "pass1 ld out", 1: "ph0 go", 2: "ph0 done",
         3: "fill1 out", 4: "ph1 go", 5: "compute end", 6: "pass1 go", 7: "end"}
# the double-buffered phases (k_grad_lds DB, batches of > 16,384 rows): slots 2
# and 3 are phases 2 and 3 going (slot 10 is then unused)
# the row-round kernel (k_grad_rt, the default for product-margin batches)
SLOTS_RT = {0: "start", 1: "issued", **{2 + t: f"round {t} go" for t in range(8)}, 10: "rounds done",
            11: "col sums done", 12: "pass1 go", 13: "end"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--features", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lds", action="store_true", help="time k_grad_lds (DLR_GRAD_RT=0) instead of k_grad_rt")
    a = ap.parse_args()
    global SLOTS
    if a.lds:
        os.environ["DLR_GRAD_RT"] = "0"
    else:
        SLOTS = SLOTS_RT
    assert "stamps" in dlr.LIB_PATH, dlr.LIB_PATH
    f = dlr.lib.dlr_debug_stamp_buffer
    f.argtypes, f.restype = [C.c_void_p], C.c_int
    D = a.features
    G = (D + 4095) // 4096
    # room for every workgroup of the launch: the fused margin may add
    # block-only workgroups past the G slices (one per CU at most)
    buf = torch.zeros(1024 * 16, dtype=torch.int64, device="cuda")
    assert f(buf.data_ptr()) == 0
    ds = dlr.Dataset.generate(a.rows, D, 50, value_mode=1, seed=10, stream=1)
    eng = dlr.Engine(D)
    eng.set_weights(dlr.init_weight(D))
    nb = eng.load_train(ds, a.batch)
    print(f"layout {eng.train_layout()} product margin {eng.train_product_margin()} batches {nb} grid {G}")
    k = 0
    rel = {s: [] for s in SLOTS}
    for rep in range(a.reps + 1):
        for _ in range(a.steps):
            eng.train_step(k % nb, 0.2, 1.0)
            k += 1
        eng.sync()
        torch.cuda.synchronize()
        st = buf[:G * 16].cpu().numpy().reshape(G, 16).astype(np.float64)
        if rep == 0:
            continue  # warm-up
        t0 = st[:, 11].min() if a.lds and st[:, 11].min() > 0 else st[:, 0].min()  # the fused margin's start
        for s in SLOTS:
            if st[:, s].min() > 0:
                rel[s].append((st[:, s] - t0) * 0.01)
    print(os.path.basename(dlr.LIB_PATH))
    print(f"{a.reps} launches, us from the first workgroup's start (percentiles over {G} workgroups)")
    for s, nm in SLOTS.items():
        if not rel[s]:
            continue
        v = np.concatenate(rel[s])
        print("  %-12s min %6.2f  p10 %6.2f  med %6.2f  p90 %6.2f  max %6.2f" % (
            nm, v.min(), np.percentile(v, 10), np.median(v), np.percentile(v, 90), v.max()))
    # the step itself (margin + this kernel + the boundaries): K steps between two syncs
    import time
    for _ in range(3):
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(500):
            eng.train_step(k % nb, 0.2, 1.0)
            k += 1
        eng.sync()
        print("  step %.2f us (500 steps, wall)" % ((time.perf_counter() - t0) / 500 * 1e6))
    eng.close()


if __name__ == "__main__":
    main()
