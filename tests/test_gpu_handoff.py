"""In-launch hand-offs: safe or loud (VERDICT r4 "Next round" 1).

Three kernels hand data from producers to consumers inside one launch: the
one-launch C2 step (k_grad_lds MG: margin blocks summed by one CU, their
residuals consumed by every CU), K6r (k_dense_ref: margin units -> column
chains) and k_band_hot (product waves -> the chain wave).  The reference's
worker never computes on data it has not received (lr.cc:122, 131:
kv_->Wait), so here

* a launch whose workgroups wait for each other is never larger than what
  the device holds at once -- the one-launch step falls back to a separate
  pass 2 when it would be (D = 2^21: 512 column slices on 256 CUs), and the
  results stay bitwise the oracle's;
* a wait whose producer never comes is bounded (250 ms) and LOUD: the step
  fails with DLR_E_DEVICE (dlr_sync / dlr_get_weights / the next
  dlr_train_step) instead of returning weights.  dlr_set_fault (test only)
  withholds one producer to prove it.
"""
from __future__ import annotations

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from test_gpu_parity import assert_same_weights

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [65536, 20000])
def test_mg_more_slices_than_cus_bitwise(B):
    # D = 2^21: 512 slices of 4,096 columns, one 1,024-thread workgroup per
    # CU -> more workgroups than are resident on MI355X's 256 CUs: the
    # one-launch margin (kind 3) must not be used; pass 2 runs in its own
    # launch (kind 2).  An epoch (the last batch wraps) + a step, bitwise.
    D = 1 << 21
    n = 150_000
    ds = dlr.Dataset.generate(n, D, 50, value_mode=1, seed=5, stream=2)
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w)
        nb = eng.load_train(ds, B)
        assert eng.train_layout() == dlr.LAYOUT_LDS
        assert eng.train_product_margin() == 2, "512 co-waiting workgroups do not fit 256 CUs"
        for b in range(nb + 1):
            eng.train_step(b % nb, 0.2, 1.0)
            g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b % nb), w)
            oracle.server_update(w, [g], 0.2)
        assert_same_weights(eng.get_weights(), w)
    finally:
        eng.close()


def _expect_device_error(fn):
    with pytest.raises(dlr.DLRError) as ei:
        fn()
    assert ei.value.code == dlr.E_DEVICE, str(ei.value)
    assert "in-launch wait ran out" in str(ei.value)
    return str(ei.value)


@pytest.mark.parametrize("B", [20_000, 16_384])
def test_mg_withheld_block_raises_then_reload_recovers(B):
    # the one-launch step (kind 3) at D = 2^20 (256 slices: resident); margin
    # block 0 never publishes -> every CU's phase-0 wait runs out -> the
    # step's weights are never returned.  B = 16,384: the row-round gradient
    # (k_grad_rt MG), whose wave 0 waits for every round's blocks.
    D = 1 << 20
    n = 45_000
    ds = dlr.Dataset.generate(n, D, 20, value_mode=1, seed=9, stream=1)
    rp, col, val, lab = ds.csr()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        nb = eng.load_train(ds, B)
        assert eng.train_product_margin() == 3
        eng.set_fault(dlr.FAULT_MG_PUBLISH)
        eng.train_step(0, 0.2, 1.0)
        msg = _expect_device_error(eng.sync)
        assert "fused margin" in msg
        _expect_device_error(lambda: eng.get_weights())
        _expect_device_error(lambda: eng.train_step(1, 0.2, 1.0))  # sticky until the next load
        # a reload clears it (and the fault: dlr_set_fault lasts one shard);
        # the context no longer trusts its one-launch step -- pass 2 runs in
        # its own launch (kind 2) -- and the steps are bitwise
        eng.set_weights(w0)
        nb = eng.load_train(ds, B)
        assert eng.train_product_margin() == 2
        w = w0.copy()
        for b in range(nb):
            eng.train_step(b, 0.2, 1.0)
            g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b), w)
            oracle.server_update(w, [g], 0.2)
        assert_same_weights(eng.get_weights(), w)
        assert eng.stage_counters()["mg_demoted"] == nb
    finally:
        eng.close()
    # a fresh context still takes the one-launch step
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        eng.load_train(ds, B)
        assert eng.train_product_margin() == 3
    finally:
        eng.close()


def test_two_engines_concurrent_c2_shape():
    # two single-rank engines on GPU 0, stepping at once
    # from two threads at the C2 shape (D = 2^20, B = 65,536: the one-launch
    # step, one 1,024-thread workgroup per CU on every CU).  Each grid needs
    # the whole device; the engine queues a co-waiting launch after the last
    # one another stream queued (CowaitScope), so neither waits on CUs the
    # other holds: both bitwise vs the oracle, no DLR_E_DEVICE.
    import threading
    D, B, nb, epochs = 1 << 20, 65_536, 3, 2
    n = nb * B
    shards = [dlr.Dataset.generate(n, D, 50, value_mode=1, seed=21 + k, stream=1) for k in range(2)]
    w0 = dlr.init_weight(D)
    engines = [dlr.Engine(D) for _ in range(2)]
    out, errs = [None, None], []
    start = threading.Barrier(2)

    def run(k):
        try:
            eng = engines[k]
            eng.set_weights(w0)
            assert eng.load_train(shards[k], B) == nb
            assert eng.train_product_margin() == 3
            start.wait(timeout=600)
            for _ in range(epochs):
                for b in range(nb):
                    eng.train_step(b, 0.2, 1.0)
            eng.sync()
            out[k] = (eng.get_weights(), eng.stage_counters())
        except BaseException as e:  # noqa: BLE001 (reported below)
            errs.append(e)
            start.abort()

    try:
        ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=900)
        assert not errs, errs
        for k in range(2):
            rp, col, val, lab = shards[k].csr()
            w = w0.copy()
            for _ in range(epochs):
                for b in range(nb):
                    g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b), w)
                    oracle.server_update(w, [g], 0.2)
            assert_same_weights(out[k][0], w)
        # the second engine's first one-launch step at least was ordered
        # behind the other's
        assert out[0][1]["cowait_serialised"] + out[1][1]["cowait_serialised"] >= 1, (out[0][1], out[1][1])
        assert out[0][1]["mg_demoted"] == 0 and out[1][1]["mg_demoted"] == 0
    finally:
        for eng in engines:
            eng.close()


def test_dense_ref_withheld_unit_raises():
    # K6r (reference-order dense step, one launch): margin unit 0 never adds
    # to its chain slot's counter -> the chains' wait for slot 0 runs out
    D, n, B = 512, 70_000, 65_536
    ds = dlr.DenseDataset.generate(n, D, seed=4, stream=1)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train_dense(ds, B)
        eng.set_fault(dlr.FAULT_REF_PUBLISH)
        eng.train_step(0, 0.2, 1.0)
        msg = _expect_device_error(eng.sync)
        assert "k_dense_ref" in msg
        _expect_device_error(lambda: eng.train_step(1, 0.2, 1.0))
    finally:
        eng.close()


def test_band_hot_withheld_ring_raises(monkeypatch):
    # k_band_hot (reference order, band mode): the product waves never post
    # a chunk -> the chain wave's wait runs out (three bands of 256 rows)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "classic")
    monkeypatch.setenv("DLR_BAND_ROWS", "256")
    monkeypatch.setenv("DLR_BAND_HOT", "32")
    D = 400
    ds = dlr.Dataset.generate(700, D, 40, value_mode=2, seed=37, stream=3)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, -1)
        assert eng.train_band_rows() == 256
        eng.set_fault(dlr.FAULT_HOT_RING)
        eng.train_step(0, 0.3, 1.0)
        msg = _expect_device_error(eng.sync)
        assert "k_band_hot" in msg
    finally:
        eng.close()


def test_hot_stream_withheld_ring_raises(monkeypatch):
    # k_hot_chain (the hot columns' chains over every band from the product
    # stream): its loader never posts a chunk -> the chain's wait runs out
    monkeypatch.setenv("DLR_BAND_ROWS", "8192")
    monkeypatch.setenv("DLR_BAND_HOT", "2000")
    D = 1 << 24
    ds = dlr.Dataset.generate_hashed(80_000, D, 39, seed=10, stream=1)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, -1)
        assert eng.train_hot_columns() > 0
        eng.set_fault(dlr.FAULT_HOT_RING)
        eng.train_step(0, 0.2, 1.0)
        msg = _expect_device_error(eng.sync)
        assert "k_hot_chain" in msg
    finally:
        eng.close()


def test_set_fault_rejects_unknown():
    eng = dlr.Engine(16)
    try:
        with pytest.raises(dlr.DLRError):
            eng.set_fault(99)
    finally:
        eng.close()
