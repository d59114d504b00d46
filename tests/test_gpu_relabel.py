"""Column relabeling (dlr_train_relabeled): a Zipf-skewed sparse shard's
columns are renumbered by frequency at load so the hot weights share cache
lines in the margin's gathers.  A pure renaming -- every sum keeps its
order -- so trajectories stay bitwise those of the oracle, through every
boundary that maps between the two numberings: set/get weights, the pushed
gradient and server update of the parameter-server topology, the RCCL
exchange (1-rank communicator), test shards loaded before or after the
training shard, and a later dense shard (identity numbering again)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, read_golden_json
from engine_driver import run_engine
from test_gpu_parity import assert_same_weights, compare_runs

pytestmark = pytest.mark.gpu

NAMES = ["c1_W1_B7_mean", "c1_W2_Bfull_mean", "c1_W2_B64_async", "real_W1_B33_mean"]


def _golden(name):
    meta = read_golden_json("trajectories.json")[name]
    base = os.path.join(GOLDEN, meta["dataset"])
    D = meta["D"]
    shards = [dlr.Dataset.load_libsvm(os.path.join(base, "train", f"part-00{p + 1}"), D)
              for p in range(meta["workers"])]
    test = dlr.Dataset.load_libsvm(os.path.join(base, "test", "part-001"), D)
    return meta, D, shards, test


@pytest.mark.parametrize("name", NAMES)
def test_forced_relabel_golden_trajectories(monkeypatch, name):
    monkeypatch.setenv("DLR_RELABEL", "1")
    meta, D, shards, test = _golden(name)
    res = run_engine(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                     test_interval=meta["test_interval"], mode=meta["mode"])
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]
    assert [p.astype("<f4").tobytes().hex() for p in res.pulled] == meta["pulled"]
    lines = [f"Iteration {it}, accuracy: {oracle.format_g(oracle.accuracy(c, n))}" for it, c, n, _ in res.tests]
    assert lines == meta["accuracy_lines"]


def test_forced_relabel_collectives(monkeypatch):
    monkeypatch.setenv("DLR_RELABEL", "1")
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    meta, D, shards, test = _golden("c1_W1_B7_mean")
    res = run_engine(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                     test_interval=meta["test_interval"], mode=meta["mode"])
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]


def _engine_run(eng, nb, epochs, lr):
    for _ in range(epochs):
        for b in range(nb):
            eng.train_step(b, lr)


def test_relabel_boundaries(monkeypatch):
    # test shard loaded BEFORE the training shard (remapped at the train
    # load), weights set before the load, round trips, dense after sparse
    D = 4096
    ds = dlr.Dataset.generate(3000, D, 20, value_mode=1, seed=21, stream=1)
    test = dlr.Dataset.generate(700, D, 20, value_mode=1, seed=21, stream=2)
    w0 = dlr.init_weight(D)
    runs = {}
    for rl in ("0", "1"):
        monkeypatch.setenv("DLR_RELABEL", rl)
        eng = dlr.Engine(D)
        try:
            eng.load_test(test)
            eng.set_weights(w0)
            nb = eng.load_train(ds, 500)
            assert eng.train_relabeled() == (rl == "1")
            assert_same_weights(eng.get_weights(), w0)
            _engine_run(eng, nb, 2, 0.1)
            runs[rl] = (eng.get_weights(), eng.predict()[:2], eng.worker_gradient(1))
            w = eng.get_weights()
            eng.set_weights(w)
            assert_same_weights(eng.get_weights(), w)
            if rl == "1":
                dd = dlr.DenseDataset.from_dataset(test)
                with pytest.raises(dlr.DLRError):
                    eng.load_test_dense(dd)
                # a dense training shard switches back to the original numbering
                eng.load_train_dense(dlr.DenseDataset.from_dataset(ds), 500)
                assert not eng.train_relabeled()
                assert_same_weights(eng.get_weights(), w)
                eng.load_test_dense(dd)
        finally:
            eng.close()
    assert_same_weights(runs["1"][0], runs["0"][0])
    assert runs["1"][1] == runs["0"][1]
    assert_same_weights(runs["1"][2], runs["0"][2], "pushed gradient")
    rp, col, val, lab = ds.csr()
    orc = oracle.run_worker([((rp, col, val), lab)], D, 2, 500, 0.1)
    assert_same_weights(runs["1"][0], orc.w)


def test_c3_shape_relabels_by_default():
    from test_gpu_layouts import _c3_shards
    D = 1 << 24
    shards = _c3_shards(1)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(shards[0], -1)
        assert eng.train_relabeled()
    finally:
        eng.close()
    # and a uniform shard does not
    eng = dlr.Engine(1 << 20)
    try:
        eng.load_train(dlr.Dataset.generate(5000, 1 << 20, 30, seed=3, stream=1), 1000)
        assert not eng.train_relabeled()
    finally:
        eng.close()


# ---- the LDS hot-weight margin (k_margin_hot): on by default for relabeled
# shards with D >= 8,192; the same products in the same order -> bitwise

@pytest.mark.parametrize("relabel", ["0", "1"])
@pytest.mark.parametrize("B", [7, 500, -1])
def test_hot_margin_forced_bitwise(monkeypatch, relabel, B):
    monkeypatch.setenv("DLR_MARGIN_HOT", "1")
    monkeypatch.setenv("DLR_RELABEL", relabel)
    D = 20000   # > 8,192 hot weights: rows mix LDS and global gathers
    ds = dlr.Dataset.generate(3000, D, 30, value_mode=1, seed=4, stream=1)
    eng = run_engine([ds], D, 2, B, 0.2)
    rp, col, val, lab = ds.csr()
    orc = oracle.run_worker([((rp, col, val), lab)], D, 2, B, 0.2)
    compare_runs(eng, orc)


def test_hot_margin_c3_equals_plain(monkeypatch):
    # C3-shaped hashed rows (relabeled, Zipf): hot margin on vs off
    D = 1 << 24
    ds = dlr.Dataset.generate_hashed(40_000, D, 39, seed=10, stream=1)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DLR_MARGIN_HOT", flag)
        out.append(run_engine([ds], D, 2, 4096, 0.2).w)
    assert_same_weights(out[1], out[0])


@pytest.mark.parametrize("W", [1, 2])
def test_rare_column_order_is_a_renaming(monkeypatch, W):
    # the rare columns (<= 16 entries) numbered by first occurrence
    # (DLR_RELABEL_TAIL=2, the default), among equal counts (1) or by id (0):
    # every numbering gives the same bits; at W = 2 the first occurrences
    # are reduced over the ranks, so both ranks number alike (a mismatch
    # would scramble the key-range exchange)
    from engine_driver import run_group
    D = 1 << 24
    shards = [dlr.Dataset.generate_hashed(30_000, D, 39, seed=12, stream=r + 1) for r in range(W)]
    out = {}
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("DLR_RELABEL_TAIL", mode)
        run = run_engine(shards, D, 2, 4096, 0.2) if W == 1 else run_group(shards, D, 2, 4096, 0.2)
        out[mode] = run.w
    assert_same_weights(out["1"], out["0"])
    assert_same_weights(out["2"], out["0"])
