"""GPU parity of the dense path (K6; BASELINE C4, and the reference's own
dense DataIter layout).  The default, reference summation order (row chains
and column chains, banded for large batches) -> bitwise.  The opt-in FAST
order (dlr_set_summation_order; blocked / fused gradients) is deterministic
and within the north-star bar |a-b| <= 1e-5*|b| + 1e-7 of the oracle at
small sizes; at C4's size it drifts past it (FAST_DRIFT)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, read_golden_json
from engine_driver import run_engine, run_group
from test_gpu_parity import assert_same_weights, compare_runs

pytestmark = pytest.mark.gpu


def dense_shard(dd: dlr.DenseDataset):
    X, y = dd.arrays()
    return X, y


FAST_DRIFT = (5e-5, 1e-6)  # |a - b| <= rel * |b| + abs: FAST's documented drift at C4's size, not a parity bar


def drift(got, want, what):
    """FAST at C4's size: prints the count outside the north-star bar and
    asserts the documented drift bound."""
    a, b = np.asarray(got, np.float64), np.asarray(want, np.float64)
    big = np.abs(b) >= 1e-2
    print(f"\n{what}: max rel {np.max(np.abs(a - b)[big] / np.abs(b)[big]):.3g} (|w| >= 1e-2), max abs "
          f"{np.max(np.abs(a - b)):.3g}, outside 1e-5*|b| + 1e-7: {int((np.abs(a - b) > 1e-5 * np.abs(b) + 1e-7).sum())}")
    assert np.all(np.abs(a - b) <= FAST_DRIFT[0] * np.abs(b) + FAST_DRIFT[1]), what


def within_bar(got, want):
    a, b = np.asarray(got, np.float64), np.asarray(want, np.float64)
    excess = np.abs(a - b) - (1e-5 * np.abs(b) + 1e-7)
    assert excess.max() <= 0, f"max excess {excess.max():.3g}"


@pytest.mark.parametrize("name", ["c1_W1_Bfull_mean", "c1_W1_B7_mean", "c1_W2_Bfull_mean", "c1_W2_B64_async",
                                  "real_W2_B50_mean", "real_W1_B33_mean"])
def test_golden_trajectories_dense(name):
    # the golden C1 shards densified (data_iter.h:28) -> the same bits
    meta = read_golden_json("trajectories.json")[name]
    base = os.path.join(GOLDEN, meta["dataset"])
    D = meta["D"]
    shards = [dlr.Dataset.load_libsvm(os.path.join(base, "train", f"part-00{p + 1}"), D)
              for p in range(meta["workers"])]
    test = dlr.Dataset.load_libsvm(os.path.join(base, "test", "part-001"), D)
    res = run_engine(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                     test_interval=meta["test_interval"], mode=meta["mode"], dense=True)
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]
    assert [p.astype("<f4").tobytes().hex() for p in res.pulled] == meta["pulled"]
    lines = [f"Iteration {it}, accuracy: {oracle.format_g(oracle.accuracy(c, n))}" for it, c, n, _ in res.tests]
    assert lines == meta["accuracy_lines"]


@pytest.mark.parametrize("D", [123, 256])
@pytest.mark.parametrize("B", [1, 7, 1001, 2500, -1])
def test_dense_batch_sizes_bitwise(D, B):
    # D=123: scalar loads; D=256: 16-byte loads.  B=2500 > N wraps twice.
    dd = dlr.DenseDataset.generate(1000, D, seed=5, stream=1)
    test = dlr.DenseDataset.generate(777, D, seed=5, stream=2)
    eng = run_engine([dd], D, 2, B, 0.05, test=test, test_interval=1, dense=True)
    orc = oracle.run_worker([dense_shard(dd)], D, 2, B, 0.05, test=dense_shard(test), test_interval=1, sparse=False)
    compare_runs(eng, orc)


def test_dense_forced_collectives(monkeypatch):
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    D = 256
    dd = dlr.DenseDataset.generate(600, D, seed=6, stream=1)
    eng = run_engine([dd], D, 2, 100, 0.05, dense=True)
    orc = oracle.run_worker([dense_shard(dd)], D, 2, 100, 0.05, sparse=False)
    compare_runs(eng, orc)


@pytest.mark.parametrize("W", [1, 2])
def test_dense_blocked_gradient_within_bar(monkeypatch, W):
    monkeypatch.setenv("DLR_DENSE_GRAD", "blocked")
    D = 512
    shards = [dlr.DenseDataset.generate(3000, D, seed=7, stream=r + 1) for r in range(W)]
    eng = run_engine(shards, D, 3, 1500, 0.05, dense=True, order=dlr.ORDER_FAST)
    orc = oracle.run_worker([dense_shard(s) for s in shards], D, 3, 1500, 0.05, sparse=False)
    within_bar(eng.w, orc.w)
    eng2 = run_engine(shards, D, 3, 1500, 0.05, dense=True, order=dlr.ORDER_FAST)
    assert_same_weights(eng2.w, eng.w)


def test_c4_shape_dense_steps(monkeypatch):
    # BASELINE C4: 4,096 dense features, B = 65,536, the FAST blocked
    # gradient (opt-in); rows reduced to two batches.
    # At this size the reference's own sequential fp32 gradient is ~1.4e-5
    # (relative) from exact arithmetic and moves a weight by ~3e-7 per step
    # (measured: see DESIGN.md "Dense"), so no reordered sum can match it to
    # a 1e-7 absolute floor -- which is why FAST is not the default.  What
    # FAST guarantees: its pushed gradient is at least as close to the
    # fp64-exact gradient as the reference's, and the weights drift by at
    # most FAST_DRIFT.
    monkeypatch.setenv("DLR_DENSE_GRAD", "blocked")  # the fused variant: test_fused_dense_*
    D, B = 4096, 65536
    dd = dlr.DenseDataset.generate(2 * B, D, seed=10, stream=1)
    X, y = dd.arrays()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_summation_order(dlr.ORDER_FAST)
        eng.set_weights(w0)
        assert eng.load_train_dense(dd, B) == 2
        rows = oracle.batch_rows(len(y), B, 0)
        g_eng = eng.worker_gradient(0, 1.0).astype(np.float64)
        g_ref = oracle.grad_dense(X, y, rows, w0).astype(np.float64)
        # fp64-exact gradient from the reference's own fp32 residuals
        z = np.zeros(B, np.float32)
        Xb = X[rows]
        for j in range(D):
            z = (z + (w0[j] * Xb[:, j]).astype(np.float32)).astype(np.float32)
        r = ((1.0 / (1.0 + np.exp(-z.astype(np.float64)))).astype(np.float32) - y[rows].astype(np.float32))
        G64 = (r[:, None].astype(np.float32) * Xb).astype(np.float32).astype(np.float64).sum(0)
        g64 = G64 / B + ((np.float32(1.0) * w0) / np.float32(B)).astype(np.float64)
        assert np.max(np.abs(g_eng - g64)) <= np.max(np.abs(g_ref - g64))
        w = w0.copy()
        for b in range(3):
            eng.train_step(b % 2, 0.05, 1.0)
            g = oracle.grad_dense(X, y, oracle.batch_rows(len(y), B, b % 2), w)
            oracle.server_update(w, [g], 0.05)
        drift(eng.get_weights(), w, "C4 shape, FAST blocked, 3 steps")
    finally:
        eng.close()


def test_dense_predict_counts_and_logloss():
    D = 1024
    test = dlr.DenseDataset.generate(20001, D, seed=9, stream=3)
    eng = dlr.Engine(D)
    try:
        w = (dlr.init_weight(D) - np.float32(0.5)).astype(np.float32)
        eng.set_weights(w)
        eng.load_test_dense(test)
        c, n, ll = eng.predict()
        X, y = test.arrays()
        c2, ll2 = oracle.predict_dense(X, y, w)
        assert (c, n) == (c2, 20001)
        assert abs(ll - ll2) <= 1e-9 * abs(ll2)
    finally:
        eng.close()


# Streamed residency (rows staged per batch from pinned host
# memory into two device slots): the same kernels on the same rows, so the
# trajectories are bitwise those of the device-resident shard -- through
# wrapping batches, batches longer than the shard, one full-shard batch,
# the blocked gradient and the collectives / worker entry points.
@pytest.mark.parametrize("B", [7, 300, 1000, 2500, -1])
def test_streamed_dense_bitwise(monkeypatch, B):
    D = 256
    dd = dlr.DenseDataset.generate(1000, D, seed=11, stream=1)
    test = dlr.DenseDataset.generate(333, D, seed=11, stream=2)
    monkeypatch.setenv("DLR_RESIDENCY", "device")
    ref = run_engine([dd], D, 3, B, 0.05, test=test, test_interval=1, dense=True)
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_engine([dd], D, 3, B, 0.05, test=test, test_interval=1, dense=True)
    assert_same_weights(got.w, ref.w)
    assert [(c, n) for _, c, n, _ in got.tests] == [(c, n) for _, c, n, _ in ref.tests]
    orc = oracle.run_worker([dense_shard(dd)], D, 3, B, 0.05, sparse=False)
    assert_same_weights(got.w, orc.w)


@pytest.mark.parametrize("W", [1, 2])
def test_streamed_dense_blocked_and_collectives(monkeypatch, W):
    monkeypatch.setenv("DLR_DENSE_GRAD", "blocked")
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    D = 512
    shards = [dlr.DenseDataset.generate(2000, D, seed=12, stream=r + 1) for r in range(W)]
    monkeypatch.setenv("DLR_RESIDENCY", "device")
    ref = run_engine(shards, D, 3, 700, 0.05, dense=True, order=dlr.ORDER_FAST)
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_engine(shards, D, 3, 700, 0.05, dense=True, order=dlr.ORDER_FAST)
    assert_same_weights(got.w, ref.w)


def test_residency_reporting():
    D = 128
    dd = dlr.DenseDataset.generate(500, D, seed=13, stream=1)
    eng = dlr.Engine(D)
    try:
        eng.load_train_dense(dd, 100)
        assert eng.train_residency() == dlr.RESIDENCY_DEVICE  # auto: fits in HBM
        eng.set_residency(dlr.RESIDENCY_STREAM)
        nb = eng.load_train_dense(dd, 100)
        assert eng.train_residency() == dlr.RESIDENCY_STREAM
        eng.set_weights(dlr.init_weight(D))
        for b in range(nb):
            eng.train_step(b, 0.05)
        with pytest.raises(dlr.DLRError):
            eng.stage_time(dlr.STAGE_MARGIN, 0, 2)
        eng.set_residency(dlr.RESIDENCY_DEVICE)
        eng.load_train_dense(dd, 100)  # the streamed shard is released (host rows unregistered)
        assert eng.train_residency() == dlr.RESIDENCY_DEVICE
        with pytest.raises(dlr.DLRError):
            eng.set_residency(7)
    finally:
        eng.close()


@pytest.mark.parametrize("rows,nbat", [(250_000, 4), pytest.param(1_048_576, 16, marks=pytest.mark.full)])
def test_c4_blocked_gradient_epoch(monkeypatch, rows, nbat):
    # The FAST blocked gradient over a C4-shaped epoch at B = 65,536 (250,000
    # rows = 4 batches, the last one wrapping to row 0; full: C4's 16-batch
    # epoch, DLR_FULL=1), against the oracle's
    # sequential sums step by step: the drift bound FAST_DRIFT (see
    # test_c4_shape_dense_steps -- the reference's own fp32 gradient moves a
    # weight ~3e-7 per step away from exact arithmetic); prints the count
    # outside the north-star bar.
    monkeypatch.setenv("DLR_DENSE_GRAD", "blocked")
    D, B, lr = 4096, 65536, 0.05
    dd = dlr.DenseDataset.generate(rows, D, seed=10, stream=2)
    X, y = dd.arrays()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_summation_order(dlr.ORDER_FAST)
        eng.set_weights(w0)
        nb = eng.load_train_dense(dd, B)
        assert nb == nbat
        w = w0.copy()
        worst = worst_abs = 0.0
        for b in range(nb):
            eng.train_step(b, lr, 1.0)
            g = oracle.grad_dense(X, y, oracle.batch_rows(len(y), B, b), w)
            oracle.server_update(w, [g], lr)
            a, bb = eng.get_weights().astype(np.float64), w.astype(np.float64)
            big = np.abs(bb) >= 1e-2
            worst = max(worst, float(np.max(np.abs(a - bb)[big] / np.abs(bb)[big])))
            worst_abs = max(worst_abs, float(np.max(np.abs(a - bb))))
            assert np.all(np.abs(a - bb) <= FAST_DRIFT[0] * np.abs(bb) + FAST_DRIFT[1]), f"step {b}"
        drift(eng.get_weights(), w, "C4 FAST blocked, 1 epoch")
        print(f"\nC4 blocked gradient, 1 epoch ({nb} x 65,536 rows, D 4,096): vs oracle max rel weight diff "
              f"{worst:.3g} (weights >= 1e-2), max abs diff {worst_abs:.3g}")
    finally:
        eng.close()


@pytest.mark.parametrize("D,B,N", [(512, 300, 1000), (1024, 256, 700), (2048, 1000, 1000), (4096, 600, 1500),
                                   (4096, 2000, 1500)])
def test_fused_dense_within_tolerance(monkeypatch, D, B, N):
    # FAST, DLR_DENSE_GRAD=fused: margin + blocked gradient partials in one
    # pass over X (LDS-staged); a blocked margin order -> tolerance,
    # deterministic.  Cases: chunks with a ragged tail (B % 256), wrapping
    # batches, B > N.
    monkeypatch.setenv("DLR_DENSE_GRAD", "fused")
    dd = dlr.DenseDataset.generate(N, D, seed=31, stream=1)
    got = run_engine([dd], D, 2, B, 0.05, dense=True, order=dlr.ORDER_FAST)
    orc = oracle.run_worker([dense_shard(dd)], D, 2, B, 0.05, sparse=False)
    within_bar(got.w, orc.w)
    again = run_engine([dd], D, 2, B, 0.05, dense=True, order=dlr.ORDER_FAST)
    assert_same_weights(again.w, got.w)


def test_fused_dense_c4_epoch_and_streamed(monkeypatch):
    # FAST fused at C4's shape (D = 4,096, B = 65,536) over a full epoch of
    # 8 batches, the last wrapping; then the same shard streamed from host:
    # bitwise equal; the drift from the oracle bounded by FAST_DRIFT
    monkeypatch.setenv("DLR_DENSE_GRAD", "fused")
    D, B, lr = 4096, 65536, 0.05
    dd = dlr.DenseDataset.generate(500_000, D, seed=10, stream=3)
    X, y = dd.arrays()
    w0 = dlr.init_weight(D)
    res = {}
    for residency in ("device", "stream"):
        monkeypatch.setenv("DLR_RESIDENCY", residency)
        eng = dlr.Engine(D)
        try:
            eng.set_summation_order(dlr.ORDER_FAST)
            eng.set_weights(w0)
            nb = eng.load_train_dense(dd, B)
            assert nb == 8
            for b in range(nb):
                eng.train_step(b, lr, 1.0)
            res[residency] = eng.get_weights()
        finally:
            eng.close()
    assert_same_weights(res["stream"], res["device"])
    w = w0.copy()
    for b in range(8):
        g = oracle.grad_dense(X, y, oracle.batch_rows(len(y), B, b), w)
        oracle.server_update(w, [g], lr)
    drift(res["device"], w, "C4 FAST fused, 1 epoch, lr 0.05")


def _glibc_exp():
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.exp.restype = ctypes.c_double
    libm.exp.argtypes = [ctypes.c_double]
    return libm.exp


def _fused_order_gradient(X, y, rows, w, C_=1.0, chunk=256):
    """The documented order of k_dense_fused + k_dense_combine (DESIGN.md §3
    item 3): row i's margin = 64 lane partials -- lane l sums columns
    256u + 4l .. 4l + 3 (u ascending) in order, fl32 products, from +0 --
    combined by the xor-butterfly tree (off 32 .. 1); r_i = fl32(sigma) - y_i
    (lr.cc:113, glibc exp); per 256-row chunk, G_k[j] = rows in order from
    +0; G[j] = chunks in order from +0; then lr.cc:40."""
    f32 = np.float32
    Xb = X[rows].astype(f32)
    Bn, D = Xb.shape
    parts = np.zeros((64, Bn), dtype=f32)
    for l in range(64):
        for u in range(D // 256):
            for c in range(4):
                j = 256 * u + 4 * l + c
                parts[l] = parts[l] + (w[j] * Xb[:, j]).astype(f32)
    v = parts
    for off in (32, 16, 8, 4, 2, 1):
        v = (v + v[np.arange(64) ^ off]).astype(f32)
    z = v[0]
    ex = _glibc_exp()
    sig = np.array([f32(1.0 / (1.0 + ex(-float(zi)))) for zi in z], dtype=f32)
    r = (sig - y[rows].astype(f32)).astype(f32)
    G = np.zeros(D, dtype=f32)
    for k0 in range(0, Bn, chunk):
        part = np.zeros(D, dtype=f32)
        for i in range(k0, min(k0 + chunk, Bn)):
            part = part + (r[i] * Xb[i]).astype(f32)
        G = (G + part).astype(f32)
    l2 = (f32(C_) * w).astype(f32) / f32(Bn)
    return (G.astype(np.float64) / np.float64(Bn) + l2.astype(f32).astype(np.float64)).astype(f32)


@pytest.mark.parametrize("D,B,N", [(512, 600, 1000), (4096, 300, 500)])
def test_fused_dense_order_bitwise(monkeypatch, D, B, N):
    # pins the fused pass to its documented (non-reference) order bit for
    # bit: the pushed gradient of batch 1 (wrapping when B does not divide
    # N) against a numpy restatement; ragged last chunk (600 = 2 x 256 + 88)
    monkeypatch.setenv("DLR_DENSE_GRAD", "fused")
    dd = dlr.DenseDataset.generate(N, D, seed=17, stream=1)
    X, y = dd.arrays()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_summation_order(dlr.ORDER_FAST)
        eng.set_weights(w0)
        eng.load_train_dense(dd, B)
        assert eng.summation_order() == dlr.ORDER_FAST
        got = eng.worker_gradient(1, 1.0)
    finally:
        eng.close()
    want = _fused_order_gradient(X, y, oracle.batch_rows(N, B, 1), w0)
    assert_same_weights(got, want, "fused pushed gradient")


# The banded reference-order launch (k_dense_ref, K6r: margin units and column
# chains in one launch; C4's default).  DLR_DENSE_REF=1 forces it at small
# sizes: slots of 256 rows with a ragged last slot, 32-row margin units,
# wrapping batches, batches longer than the shard, a shard shorter than a slot,
# the pushed gradient (world > 1 / parameter-server path) and streamed rows --
# all bitwise the oracle (lr.cc:35-40, 108-113).
@pytest.mark.parametrize("D,B,N", [(512, 300, 1000), (512, 1000, 700), (1024, 5000, 3000), (4096, 600, 1500),
                                   (4096, 1500, 1500), (2048, 100, 100), (512, 33, 40), (640, 4096, 9000)])
def test_dense_ref_banded_bitwise(monkeypatch, D, B, N):
    monkeypatch.setenv("DLR_DENSE_REF", "1")
    dd = dlr.DenseDataset.generate(N, D, seed=41, stream=1)
    eng = run_engine([dd], D, 2, B, 0.2, dense=True)
    orc = oracle.run_worker([dense_shard(dd)], D, 2, B, 0.2, sparse=False)
    compare_runs(eng, orc)


@pytest.mark.parametrize("W", [2, 3])
def test_dense_ref_banded_ranks(monkeypatch, W):
    # the pushed gradient (non-fused epilogue): the parameter-server topology
    # and the loopback group's key-range exchange
    monkeypatch.setenv("DLR_DENSE_REF", "1")
    D = 1024
    shards = [dlr.DenseDataset.generate(1200, D, seed=43, stream=r + 1) for r in range(W)]
    orc = oracle.run_worker([dense_shard(s) for s in shards], D, 2, 700, 0.2, sparse=False)
    got = run_engine(shards, D, 2, 700, 0.2, dense=True)
    assert_same_weights(got.w, orc.w, "parameter-server topology")
    grp = run_group(shards, D, 2, 700, 0.2, dense=True)
    assert_same_weights(grp.w, orc.w, "loopback group")


def test_dense_ref_banded_streamed(monkeypatch):
    monkeypatch.setenv("DLR_DENSE_REF", "1")
    D = 2048
    dd = dlr.DenseDataset.generate(3000, D, seed=47, stream=1)
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_engine([dd], D, 3, 1300, 0.2, dense=True)
    orc = oracle.run_worker([dense_shard(dd)], D, 3, 1300, 0.2, sparse=False)
    assert_same_weights(got.w, orc.w)


def test_dense_ref_default_for_c4_shape():
    # the reference order picks the banded launch for C4-sized batches
    D, B = 4096, 65536
    dd = dlr.DenseDataset.generate(B + 1000, D, seed=10, stream=4)
    X, y = dd.arrays()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        assert eng.load_train_dense(dd, B) == 2 and eng.summation_order() == dlr.ORDER_REFERENCE
        w = w0.copy()
        for b in (0, 1, 1, 0):  # the second batch wraps to row 0
            eng.train_step(b, 0.2, 1.0)
            oracle.server_update(w, [oracle.grad_dense(X, y, oracle.batch_rows(len(y), B, b), w)], 0.2)
            assert_same_weights(eng.get_weights(), w, f"C4 shape, batch {b}")
    finally:
        eng.close()
