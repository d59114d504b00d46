"""Multi-step launches (dlr_train_steps, k_grad_lds_ms): LR::Train's epoch
loop (lr.cc:29-44) over one-launch steps, up to 32 of them in ONE launch --
the launch boundary between steps replaced by an in-launch hand-off of the
next batch's products.  The same steps in the same order, so every result
must be BITWISE the per-step launches (DLR_MULTI_STEP=0) and the oracle's
sparse port: across launch boundaries (32 steps each), epoch wraps, a start
mid-epoch, weights changed between calls, ragged and empty rows, a
withheld producer (loud), and two engines stepping at once."""
from __future__ import annotations

import threading

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from test_gpu_parity import assert_same_weights

pytestmark = pytest.mark.gpu


def _oracle_steps(csr, lab, n, B, w, batches, lr=0.2):
    for b in batches:
        g = oracle.grad_csr(csr, lab, oracle.batch_rows(n, B, b), w)
        oracle.server_update(w, [g], lr)
    return w


def _ragged_ds(D, n, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 65, size=n)
    lens[rng.choice(n, 3000, replace=False)] = 0
    lens[64 * 40:64 * 42] = 0  # two empty 64-row blocks
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(D, k, replace=False)) for k in lens]).astype(np.int32)
    val = rng.integers(1, 10001, size=len(col)).astype(np.float32) / np.float32(10000)
    lab = rng.integers(0, 2, size=n).astype(np.int32)
    return dlr.Dataset.from_csr(rp, col, val, lab, D)


def test_multi_step_c2_shape_bitwise(monkeypatch):
    # BASELINE C2's shape (D = 10^6: 245 slices, B = 65,536: one launch
    # per step) over 4 batches (the last wraps): 70 steps from batch 0 =
    # launches of 32 + 32 + 6 steps crossing 17 epoch boundaries, then 5
    # steps from batch 2 (the products of the first are formed first)
    D, B, n = 1_000_000, 65_536, 200_000
    ds = dlr.Dataset.generate(n, D, 50, value_mode=1, seed=12, stream=1)
    rp, col, val, lab = ds.csr()
    w0 = dlr.init_weight(D)

    def run(ms):
        monkeypatch.setenv("DLR_MULTI_STEP", ms)
        eng = dlr.Engine(D)
        try:
            eng.set_weights(w0)
            nb = eng.load_train(ds, B)
            assert eng.train_product_margin() == 3
            assert eng.train_multi_step() == (ms == "1")
            eng.train_steps(0, 70, 0.2, 1.0)
            mid = eng.get_weights()
            eng.train_steps(2, 5, 0.2, 1.0)
            return mid, eng.get_weights(), nb
        finally:
            eng.close()

    (mid, end, nb), (rmid, rend, _) = run("1"), run("0")
    assert_same_weights(mid, rmid)
    assert_same_weights(end, rend)
    w = _oracle_steps((rp, col, val), lab, n, B, w0.copy(), [b % nb for b in range(70)])
    assert_same_weights(mid, w)
    w = _oracle_steps((rp, col, val), lab, n, B, w, [(2 + k) % nb for k in range(5)])
    assert_same_weights(end, w)


@pytest.mark.parametrize("B", [20_000, 40_000])
def test_multi_step_ragged_interleaved(monkeypatch, B):
    # ragged rows (empty rows and blocks), fewer slices than CUs (the
    # evened grid's block-only workgroups take part in every step's
    # hand-off), single steps and set_weights between multi-step calls
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    D, n = 1 << 20, 100_000
    ds = _ragged_ds(D, n, 31)
    rp, col, val, lab = ds.csr()
    w0 = dlr.init_weight(D)
    bump = np.random.default_rng(3).standard_normal(D).astype(np.float32) * np.float32(0.01)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        nb = eng.load_train(ds, B)
        assert eng.train_product_margin() == 3 and eng.train_multi_step()
        w = w0.copy()
        eng.train_steps(1, 9, 0.2, 1.0)
        w = _oracle_steps((rp, col, val), lab, n, B, w, [(1 + k) % nb for k in range(9)])
        eng.train_step(0, 0.2, 1.0)  # a step the last launch did not guess
        w = _oracle_steps((rp, col, val), lab, n, B, w, [0])
        eng.set_weights(eng.get_weights() + bump)
        w = w + bump
        eng.train_steps(1, 40, 0.2, 1.0)
        w = _oracle_steps((rp, col, val), lab, n, B, w, [(1 + k) % nb for k in range(40)])
        eng.train_epoch(0.2, 1.0)
        w = _oracle_steps((rp, col, val), lab, n, B, w, list(range(nb)))
        assert_same_weights(eng.get_weights(), w)
    finally:
        eng.close()


def test_multi_step_withheld_block_raises_then_demotes():
    # margin block 0 of the first step never publishes: every workgroup's
    # wait runs out (once: the launch's later waits end at once), the call
    # is loud, and the context's next load runs separate launches (kind 2)
    D, B, n = 1 << 20, 20_000, 45_000
    ds = dlr.Dataset.generate(n, D, 20, value_mode=1, seed=9, stream=1)
    rp, col, val, lab = ds.csr()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        nb = eng.load_train(ds, B)
        assert eng.train_multi_step()
        eng.set_fault(dlr.FAULT_MG_PUBLISH)
        eng.train_steps(0, 12, 0.2, 1.0)
        with pytest.raises(dlr.DLRError) as ei:
            eng.sync()
        assert ei.value.code == dlr.E_DEVICE and "fused margin" in str(ei.value)
        eng.set_weights(w0)
        nb = eng.load_train(ds, B)
        assert eng.train_product_margin() == 2 and not eng.train_multi_step()
        eng.train_steps(0, 2 * nb, 0.2, 1.0)
        w = _oracle_steps((rp, col, val), lab, n, B, w0.copy(), [b % nb for b in range(2 * nb)])
        assert_same_weights(eng.get_weights(), w)
    finally:
        eng.close()


def test_multi_step_two_engines_concurrent():
    # two engines' multi-step launches at once from two threads, each grid
    # one workgroup per CU on every CU for up to 32 steps: ordered one
    # after the other (CowaitScope), both bitwise
    D, B, nb = 1 << 20, 65_536, 3
    n = nb * B
    shards = [dlr.Dataset.generate(n, D, 50, value_mode=1, seed=41 + k, stream=1) for k in range(2)]
    w0 = dlr.init_weight(D)
    engines = [dlr.Engine(D) for _ in range(2)]
    out, errs = [None, None], []
    start = threading.Barrier(2)

    def run(k):
        try:
            eng = engines[k]
            eng.set_weights(w0)
            eng.load_train(shards[k], B)
            assert eng.train_multi_step()
            start.wait(timeout=600)
            for _ in range(3):
                eng.train_steps(0, 2 * nb, 0.2, 1.0)
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
            w = _oracle_steps((rp, col, val), lab, n, B, w0.copy(), [b % nb for b in range(6 * nb)])
            assert_same_weights(out[k][0], w)
        assert out[0][1]["cowait_serialised"] + out[1][1]["cowait_serialised"] >= 1
    finally:
        for eng in engines:
            eng.close()
