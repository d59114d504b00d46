"""Diagnosis: per-batch worker gradients of the ragged-rows case vs the oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dist-lr_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import distlr_amd as dlr, oracle
from parse_format import csr_to_dense

rng = np.random.default_rng(7)
D, n = 700, 3000
lens = rng.integers(0, 60, size=n)
lens[rng.choice(n, 300, replace=False)] = 0
lens[5] = 700
rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
col = np.concatenate([np.sort(rng.choice(D, k, replace=False)) for k in lens]).astype(np.int32)
val = rng.integers(1, 10001, size=len(col)).astype(np.float32) / np.float32(10000)
lab = rng.integers(0, 2, size=n).astype(np.int32)
ds = dlr.Dataset.from_csr(rp, col, val, lab, D)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 257
w0 = dlr.init_weight(D)
eng = dlr.Engine(D)
eng.set_weights(w0)
nb = eng.load_train(ds, B)
bad = 0
for b in range(nb):
    g = eng.worker_gradient(b, 1.0)
    go = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b), w0)
    d = np.nonzero(g.view(np.uint32) != go.view(np.uint32))[0]
    if len(d):
        bad += 1
        rows = oracle.batch_rows(n, B, b)
        print(f"batch {b}: {len(d)} cols differ, first {d[:8]}, rows {rows[0]}..{rows[-1]}, "
              f"maxrel {np.max(np.abs(g[d]-go[d])/np.maximum(np.abs(go[d]),1e-30)):.3g}")
print(f"SEG={os.environ.get('DLR_MARGIN_SEG','auto')} B={B}: {bad} of {nb} batches differ")

# Step-by-step trajectory: fused train_step vs oracle.
eng.set_weights(w0)
w = w0.copy()
for ep in range(3):
    for b in range(nb):
        wprev = w.copy()
        eng.train_step(b, 0.3, 1.0)
        go = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b), wprev)
        oracle.server_update(w, [go], 0.3)
        wg = eng.get_weights()
        d = np.nonzero(wg.view(np.uint32) != w.view(np.uint32))[0]
        if len(d):
            print(f"epoch {ep} batch {b}: {len(d)} weights differ first {d[:6]}")
            # recompute the step's gradient on the GPU from the same start
            eng.set_weights(wprev)
            g2 = eng.worker_gradient(b, 1.0)
            dg = np.nonzero(g2.view(np.uint32) != go.view(np.uint32))[0]
            print(f"   worker_gradient from the same start: {len(dg)} cols differ {dg[:6]}")
            j = d[0]
            print(f"   w[{j}] gpu {wg[j]!r} oracle {w[j]!r} prev {wprev[j]!r} g_gpu {g2[j]!r} g_orc {go[j]!r}")
            print("   fused check:", np.float32(wprev[j]) - np.float32(np.float32(0.3) * go[j]))
            sys.exit(0)
print("trajectory: identical for 3 epochs")
