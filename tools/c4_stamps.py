#!/usr/bin/env python3
"""Per-workgroup timeline of the banded reference-order dense launch
(k_dense_ref, C4) from s_memrealtime stamps (100 MHz).  Loads the DLR_STAMPS
build of the library (make -C dist-lr_amd stamps) through DLR_LIB.
Development tool, never part of the product.

Chain halves (row b of the buffer): 0 start, 2 + t/16 the end of slot t's
chain (t = 0, 16, ...), 50 end; totals (us): 52 / 53 the chain wave waiting
for the helpers / adding, 54 / 55 / 56 helper 1 waiting for residuals / for
the chain / transforming and issuing loads, 57 / 58 wave 3 waiting for the
margins / for the helpers; 60-63 s_memtime / s_memrealtime at the chain's
start and end (the shader clock under load).  Margin halves (row 256 + b): 1 first claims
done, 2 + k the publish time of its k-th unit, 22 + k its start (after the
limit), 42 + k its id (k < 20), 63 end; totals over the launch (us): 60 the
compute wave waiting for stages, 61 adding; loaders 0 / 1: 56 / 58 issuing
(including the waits for ring slots and unit ids), 57 / 59 waiting for
their DMA to land.

  python tools/c4_stamps.py [--rows N] [--steps K] [--reps R]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_abl = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--abl=")), "0")
_n, _, _v = _abl.partition("_")  # "N" or "N_name": make stamps ABL=N [SVAR=name]
os.environ.setdefault("DLR_LIB", os.path.join(ROOT, "dist-lr_amd", "lib", "libdistlr_amd_stamps%s%s.so" % (
    "" if _n == "0" else "_abl" + _n, "_" + _v if _v else "")))
sys.path.insert(0, os.path.join(ROOT, "dist-lr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (one HIP runtime: torch's)

import distlr_amd as dlr  # noqa: E402


def pct(v):
    v = np.asarray(v, dtype=np.float64)
    if v.size == 0:
        return "(none)"
    return "min %7.1f p10 %7.1f med %7.1f p90 %7.1f max %7.1f" % tuple(np.percentile(v, [0, 10, 50, 90, 100]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=300_000)
    ap.add_argument("--features", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--abl", default="0",
                    help="ablation / variant build: --abl=N (make stamps ABL=N), --abl=N_name (SVAR=name)")
    ap.add_argument("--lead", type=int, default=None, help="DLR_DENSE_REF_LEAD (0: no limit)")
    a = ap.parse_args()
    if a.lead is not None:
        os.environ["DLR_DENSE_REF_LEAD"] = str(a.lead)
    assert "stamps" in dlr.LIB_PATH, dlr.LIB_PATH
    f = dlr.lib.dlr_debug_stamp_buffer
    f.argtypes, f.restype = [C.c_void_p], C.c_int
    D, B = a.features, a.batch
    S = D // 16
    M = min(256, (B + 63) // 64)
    G = 512  # chain workgroups write rows [0, S), margin workgroups rows [256, 256 + M)
    buf = torch.zeros(G * 64, dtype=torch.int64, device="cuda")
    assert f(buf.data_ptr()) == 0
    dd = dlr.DenseDataset.generate(a.rows, D, seed=10, stream=1)
    eng = dlr.Engine(D)
    eng.set_weights(dlr.init_weight(D))
    nb = eng.load_train_dense(dd, B)
    nslot = (B + 255) // 256
    k = 0
    for rep in range(a.reps + 1):
        buf.zero_()
        torch.cuda.synchronize()
        for _ in range(a.steps):
            eng.train_step(k % nb, 0.2, 1.0)
            k += 1
        eng.sync()
        torch.cuda.synchronize()
        st = buf.cpu().numpy().reshape(G, 64).astype(np.float64)
        if rep == 0:
            continue  # warm-up
        ch, mg = st[:S], st[256:256 + M]
        t0 = ch[:, 0].min()
        us = lambda x: (x - t0) * 0.01  # noqa: E731
        print(f"--- last launch of rep {rep}: {S} chain + {M} margin workgroups, {nslot} slots")
        print("chain start      ", pct(us(ch[:, 0])))
        for t in range(0, nslot + 1, 32):
            print(f"chain slot {t:4d}  ", pct(us(ch[:, 2 + t // 16])))
        print("chain end        ", pct(us(ch[:, 50])))
        ctick = lambda c: pct(ch[:, c] * 0.01)  # noqa: E731
        print("chain: waiting for helpers ", ctick(52))
        print("chain: adding              ", ctick(53))
        print("helper 1: waiting residuals", ctick(54))
        print("helper 1: waiting the chain", ctick(55))
        print("helper 1: transform + loads", ctick(56))
        print("wave 3: waiting margins    ", ctick(57))
        print("wave 3: waiting helpers    ", ctick(58))
        ghz = (ch[:, 62] - ch[:, 60]) / np.maximum(1.0, (ch[:, 63] - ch[:, 61])) * 0.1
        print("shader clock over the chain (GHz)", pct(ghz))
        print("margin claims    ", pct(us(mg[:, 1])))
        ids = []
        for kk in range(20):
            m = mg[:, 2 + kk] > 0
            if not m.any():
                break
            st_, pu = us(mg[m, 22 + kk]), us(mg[m, 2 + kk])
            print(f"margin unit #{kk:2d} start", pct(st_), f"({m.sum()} WGs)")
            print(f"              busy ", pct(pu - st_))
            ids += list(zip(mg[m, 42 + kk], pu))
        print("margin end       ", pct(us(mg[:, 63])))
        tick = lambda c: pct(mg[:, c] * 0.01)  # noqa: E731
        print("compute: waiting for stages", tick(60))
        print("compute: adding            ", tick(61))
        print("loader 0: issuing          ", tick(56))
        print("loader 0: waiting to land  ", tick(57))
        print("loader 1: issuing          ", tick(58))
        print("loader 1: waiting to land  ", tick(59))
        ids.sort()
        if ids:
            u = np.array([x for x, _ in ids])
            t = np.array([y for _, y in ids])
            slots = u // 4
            print("slot publish time (last unit of slot):")
            for s_ in range(0, nslot, 32):
                m = slots == s_
                if m.any():
                    print(f"   slot {s_:4d}: {t[m].max():8.1f} us")
        print(f"wall per step (bench-style) n/a; chain span {np.median(us(ch[:, 50])):.1f} us")


if __name__ == "__main__":
    main()
