"""Unit-valued shards (dlr_train_unit_values): when every value of a sparse
shard is exactly 1.0f (a9a / gen_data.py's C1 data, Criteo-style hashed
fields, BASELINE C3 and C5) the engine stores no value arrays and runs the
kernels' UNIT variants, which never read values.  fl32(t * 1.0f) == t, so
every result must be bitwise that of the valued path (DLR_UNIT_VALUES=0):
per gradient layout, through the chunked long columns of a C3-shaped shard
(whose padding entries the UNIT path must skip), the RCCL exchange, the
pushed gradient and prediction."""
from __future__ import annotations

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from engine_driver import run_engine
from test_gpu_parity import assert_same_weights
from test_gpu_relabel import _golden

pytestmark = pytest.mark.gpu


def test_unit_detection(monkeypatch):
    _, D, shards, test = _golden("c1_W1_B7_mean")
    _, Dr, real, _ = _golden("real_W1_B33_mean")
    sizes = {}
    for env in ("1", "0"):
        monkeypatch.setenv("DLR_UNIT_VALUES", env)
        with dlr.Engine(D) as eng:
            eng.load_train(shards[0], 7)
            assert eng.train_unit_values() == (env == "1")
            sizes[env] = eng.memory_info()[0]
        with dlr.Engine(Dr) as eng:
            eng.load_train(real[0], 33)
            assert not eng.train_unit_values()
    assert sizes["1"] < sizes["0"]
    # one value off 1.0f: the valued path
    rp, col, val, lab = shards[0].csr()
    val = val.copy()
    val[len(val) // 2] = np.float32(1.0000001)
    ds = dlr.Dataset.from_csr(rp, col, val, lab, D)
    monkeypatch.delenv("DLR_UNIT_VALUES")
    with dlr.Engine(D) as eng:
        eng.set_weights(dlr.init_weight(D))
        nb = eng.load_train(ds, 7)
        assert not eng.train_unit_values()
        for b in range(nb):
            eng.train_step(b, 0.2)
        w = eng.get_weights()
    orc = oracle.run_worker([((rp, col, val), lab)], D, 1, 7, 0.2)
    assert_same_weights(w, orc.w)


@pytest.mark.parametrize("layout", ["classic", "lds", "touched"])
@pytest.mark.parametrize("name", ["c1_W1_B7_mean", "c1_W2_B64_async"])
def test_valued_path_golden_per_layout(monkeypatch, layout, name):
    # the golden trajectories (unit data) with the value arrays kept: the
    # default runs take the UNIT path in test_gpu_parity / test_gpu_layouts
    monkeypatch.setenv("DLR_UNIT_VALUES", "0")
    monkeypatch.setenv("DLR_GRAD_KERNEL", layout)
    meta, D, shards, test = _golden(name)
    try:
        res = run_engine(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                         test_interval=meta["test_interval"], mode=meta["mode"])
    except dlr.DLRError as e:
        if "do not fit the LDS layout" in str(e):
            pytest.skip("batches too dense for the LDS layout")
        raise
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]
    lines = [f"Iteration {it}, accuracy: {oracle.format_g(oracle.accuracy(c, n))}" for it, c, n, _ in res.tests]
    assert lines == meta["accuracy_lines"]


def _c3(W, rows=60_000):
    return [dlr.Dataset.generate_hashed(rows, 1 << 24, 39, seed=10, stream=r + 1) for r in range(W)]


@pytest.mark.parametrize("W", [1, 2])
def test_c3_unit_long_columns_equal_valued(monkeypatch, W):
    # chunked long columns (default) with their padding entries: UNIT and
    # valued give the same bits, including the rank-ordered W = 2 merge
    D = 1 << 24
    shards = _c3(W)
    runs = {}
    for env in ("0", "1"):
        monkeypatch.setenv("DLR_UNIT_VALUES", env)
        runs[env] = run_engine(shards, D, 3, -1, 0.2)
    assert_same_weights(runs["1"].w, runs["0"].w)


def test_c3_unit_gradient_and_collectives(monkeypatch):
    D = 1 << 24
    ds = _c3(1)[0]
    w0 = dlr.init_weight(D)
    out = {}
    for env in ("0", "1"):
        monkeypatch.setenv("DLR_UNIT_VALUES", env)
        with dlr.Engine(D) as eng:
            eng.set_weights(w0)
            eng.load_train(ds, -1)
            assert eng.train_unit_values() == (env == "1")
            out[env] = eng.worker_gradient(0, 1.0)
    assert_same_weights(out["1"], out["0"], "pushed gradient")
    monkeypatch.setenv("DLR_UNIT_VALUES", "1")
    ref = run_engine([ds], D, 2, -1, 0.2)
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    got = run_engine([ds], D, 2, -1, 0.2)
    assert_same_weights(got.w, ref.w)


def test_unit_predict(monkeypatch):
    meta, D, shards, test = _golden("c1_W1_Bfull_mean")
    res = {}
    for env in ("0", "1"):
        monkeypatch.setenv("DLR_UNIT_VALUES", env)
        with dlr.Engine(D) as eng:
            eng.set_weights(dlr.init_weight(D))
            nb = eng.load_train(shards[0], -1)
            eng.load_test(test)
            for b in range(nb):
                eng.train_step(b, 0.2)
            res[env] = eng.predict()
    assert res["1"] == res["0"]
