"""Full-size parity of the reference summation orders, and the world > 1
engine path at the north-star shapes ("Next round" items 1 and 3).

* C3 (12.5M-row Criteo-shaped shard, B = -1) in the reference summation
  order (the default, dlr_set_summation_order): every column is ONE
  sequential fp32 sum in batch-row order (lr.cc:35-39), carried across the
  2^20-row bands -> the weights after each of two steps are BITWISE the
  oracle's, with the centred init whose residuals are general fp32 values
  (the FAST long-column phase tree: test_gpu_c3_full.py).
* C4 (D = 4,096, B = 65,536) in the reference order at the bench's lr 0.2:
  a full epoch of 16 batches (the last wrapping to row 0), bitwise after
  every step (margin: one chain per row in column order, lr.cc:108-112;
  gradient: one chain per column in row order, lr.cc:35-39).
* W = 8 ranks on the loopback group at C3's structure with 2.2M-row shards
  (the default 2^20-row bands apply from 2^21 rows): relabeling from the
  summed counts, bands, hot-weight margin, key-range all-to-all of 2^24
  weights over 8 ranks (main.cc:57-78's merge in rank order), 2 steps --
  bitwise in the reference order, within 1e-5*|b| + 1e-7 under FAST.
* C4's shape (D = 4,096, B = 65,536) on W = 2 and W = 4 loopback ranks:
  bitwise in the reference order at lr 0.2; the FAST fused variant's
  deviation at lr 0.2 is measured against the north-star bar and printed
  (it exceeds it: FAST is opt-in).
"""
from __future__ import annotations

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from engine_driver import run_group
from test_gpu_parity import assert_same_weights

pytestmark = pytest.mark.gpu


def within_bar(got, want, what=""):
    # BASELINE.md's bar: 1e-5 relative with a 1e-7 absolute floor
    a, b = got.astype(np.float64), want.astype(np.float64)
    bad = np.abs(a - b) > 1e-5 * np.abs(b) + 1e-7
    assert not bad.any(), f"{what}: {int(bad.sum())} weights outside 1e-5*|b| + 1e-7"


def test_c3_full_size_reference_order_bitwise():
    D, ROWS, LR = 1 << 24, 12_500_000, 0.2
    ds = dlr.Dataset.generate_hashed(ROWS, D, 39, seed=10, stream=1)
    rp, col, val, lab = ds.csr()
    csr = (rp, col, val)
    rows = oracle.batch_rows(ROWS, -1, 0)
    w0 = dlr.init_weight(D)
    w0 = ((w0 - np.float32(0.5)) / np.float32(5.0)).astype(np.float32)  # centred: general fp32 residuals
    assert np.bincount(col, minlength=D).max() > 500_000  # the ~10^6-entry chains are there
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        assert eng.load_train(ds, -1) == 1
        assert eng.train_band_rows() == 1 << 19 and eng.train_relabeled()  # REFERENCE: half-size bands
        assert eng.summation_order() == dlr.ORDER_REFERENCE
        w = w0.copy()
        for step in range(2):
            eng.train_step(0, LR, 1.0)
            oracle.server_update(w, [oracle.grad_csr(csr, lab, rows, w)], LR)
            assert_same_weights(eng.get_weights(), w, f"C3 reference order, step {step}")
    finally:
        eng.close()


def test_c4_full_epoch_reference_order_bitwise():
    D, B, lr = 4096, 65536, 0.2
    dd = dlr.DenseDataset.generate(1_000_000, D, seed=10, stream=2)
    X, y = dd.arrays()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        nb = eng.load_train_dense(dd, B)
        assert nb == 16 and eng.summation_order() == dlr.ORDER_REFERENCE
        w = w0.copy()
        for b in range(nb):
            eng.train_step(b, lr, 1.0)
            oracle.server_update(w, [oracle.grad_dense(X, y, oracle.batch_rows(len(y), B, b), w)], lr)
            assert_same_weights(eng.get_weights(), w, f"C4 reference order, step {b}")
    finally:
        eng.close()


def _c3_shards(W, rows):
    return [dlr.Dataset.generate_hashed(rows, 1 << 24, 39, seed=10, stream=r + 1) for r in range(W)]


def _csr(ds):
    rp, col, val, lab = ds.csr()
    return (rp, col, val), lab


@pytest.fixture(scope="module")
def c3_w8():
    shards = _c3_shards(8, 2_200_000)
    return shards, [_csr(s) for s in shards]


@pytest.mark.parametrize("order", ["reference", "fast"])
def test_c3_eight_ranks_loopback(c3_w8, order):
    shards, csrs = c3_w8
    o = dlr.ORDER_REFERENCE if order == "reference" else dlr.ORDER_FAST
    D = 1 << 24
    eng = dlr.Engine(D)
    try:  # the choices at this shard size (one rank's view)
        eng.set_summation_order(o)
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(shards[0], -1)
        assert eng.train_band_rows() == (1 << 19 if order == "reference" else 1 << 20)
        assert eng.train_relabeled() and eng.train_unit_values()
        assert eng.summation_order() == o
    finally:
        eng.close()
    got = run_group(shards, D, 2, -1, 0.2, order=o)
    orc = oracle.run_worker(csrs, D, 2, -1, 0.2)
    if order == "reference":
        assert_same_weights(got.w, orc.w, "W = 8, reference order")
    else:
        within_bar(got.w, orc.w, "W = 8, long-column phases")


@pytest.mark.parametrize("order,W", [("reference", 2), ("reference", 4), ("fast", 2),
                                     pytest.param("fast", 4, marks=pytest.mark.full)])
def test_dense_c4_shape_ranks(monkeypatch, W, order):
    # C4's shape (D = 4,096, B = 65,536; 3 batches per epoch, the last
    # wrapping) on W loopback ranks at the bench's lr 0.2.  Reference order
    # (the default: lr.cc:108-112 row chains, lr.cc:35-39 column chains):
    # bitwise.  FAST (the fused blocked pass, opt-in): it does NOT meet the
    # north-star bar here -- the test pins that it stays
    # deterministic, reports how many weights leave 1e-5*|b| + 1e-7, and
    # bounds the drift at 1e-3 relative (1e-5 absolute) so a regression is
    # still caught.
    D, B, rows, lr = 4096, 65536, 150_000, 0.2
    o = dlr.ORDER_REFERENCE if order == "reference" else dlr.ORDER_FAST
    if order == "fast":
        monkeypatch.setenv("DLR_DENSE_GRAD", "fused")
    shards = [dlr.DenseDataset.generate(rows, D, seed=10, stream=r + 5) for r in range(W)]
    arrays = [s.arrays() for s in shards]
    eng = dlr.Engine(D)
    try:
        eng.set_summation_order(o)
        eng.set_weights(dlr.init_weight(D))
        assert eng.load_train_dense(shards[0], B) == 3
        assert eng.summation_order() == o
    finally:
        eng.close()
    # (W = 4 runs one epoch -- its three batches, the last wrapping -- to
    # keep the suite's time down; FAST at W = 4 two, DLR_FULL=1)
    epochs = 2 if W == 2 or order == "fast" else 1
    got = run_group(shards, D, epochs, B, lr, dense=True, order=o)
    orc = oracle.run_worker(arrays, D, epochs, B, lr, sparse=False)
    if order == "reference":
        assert_same_weights(got.w, orc.w, f"reference order, W = {W}")
        return
    again = run_group(shards, D, epochs, B, lr, dense=True, order=o)
    assert np.array_equal(got.w.view(np.uint32), again.w.view(np.uint32)), "FAST is not deterministic"
    a, b = got.w.astype(np.float64), orc.w.astype(np.float64)
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-30)
    print(f"\nFAST fused dense, W = {W}, lr {lr}: max rel {rel[np.abs(b) >= 1e-2].max():.3g} (|b| >= 1e-2), "
          f"max abs {np.abs(a - b).max():.3g}, "
          f"outside 1e-5*|b| + 1e-7: {int((np.abs(a - b) > 1e-5 * np.abs(b) + 1e-7).sum())} of {D}")
    # the drift bound (not the north-star bar): 1e-3 relative, 1e-5 absolute
    # for the small weights
    assert np.all(np.abs(a - b) <= 1e-3 * np.abs(b) + 1e-5)
