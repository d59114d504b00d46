"""K1 for sparse shards (north_star: "coalesced CSR upload of each minibatch
from DataIter into pinned buffers with async copies"; data_iter.h:40-55 is
the surface it replaces): with DLR_RESIDENCY_STREAM the shard's CSR and its
per-batch column-major copies stay in page-locked host memory and each
batch's slices are staged into one of two device slots on the copy stream
while the previous batch computes.  The kernels are unchanged, so results
must be BITWISE those of the resident shard -- and of the oracle -- for
every layout, wrapping batches, the touched exchange and the key-range
exchange."""
from __future__ import annotations

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from engine_driver import run_engine, run_group
from test_gpu_parity import assert_same_weights, compare_runs, oracle_shard

pytestmark = pytest.mark.gpu


def _csr(ds):
    rp, col, val, lab = ds.csr()
    return (rp, col, val), lab


@pytest.mark.parametrize("layout", ["lds", "classic", "touched"])
@pytest.mark.parametrize("B", [7, 1001, 2999, -1])
def test_streamed_sparse_bitwise(monkeypatch, layout, B):
    # B = 2999 wraps twice per epoch... (3,000 rows: batches 0 and 1 contiguous, the last wraps)
    monkeypatch.setenv("DLR_GRAD_KERNEL", layout)
    D = 30000
    ds = dlr.Dataset.generate(3000, D, 20, value_mode=1, seed=21, stream=1)
    test = dlr.Dataset.generate(500, D, 20, value_mode=1, seed=21, stream=2)
    monkeypatch.setenv("DLR_RESIDENCY", "device")
    try:
        ref = run_engine([ds], D, 2, B, 0.1, test=test, test_interval=1)
    except dlr.DLRError as e:
        if "do not fit the LDS layout" in str(e):
            pytest.skip("batches too dense for the LDS layout")
        raise
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_engine([ds], D, 2, B, 0.1, test=test, test_interval=1)
    compare_runs(got, ref)
    orc = oracle.run_worker([_csr(ds)], D, 2, B, 0.1)
    assert_same_weights(got.w, orc.w)


@pytest.mark.parametrize("coalesce,device_layout", [("1", "1"), ("0", "1"), ("1", "0"), ("0", "0")])
def test_streamed_copy_paths_bitwise(monkeypatch, coalesce, device_layout):
    # one coalesced copy per batch (default) or one copy per array and batch
    # (DLR_STREAM_COALESCE=0); the LDS layout built on the device from the
    # staged CSR (default) or streamed as built on the host
    # (DLR_STREAM_DEVICE_LAYOUT=0): the same sums either way
    monkeypatch.setenv("DLR_STREAM_COALESCE", coalesce)
    monkeypatch.setenv("DLR_STREAM_DEVICE_LAYOUT", device_layout)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    D = 30000
    ds = dlr.Dataset.generate(3000, D, 20, value_mode=1, seed=23, stream=1)
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_engine([ds], D, 2, 1001, 0.1)
    orc = oracle.run_worker([_csr(ds)], D, 2, 1001, 0.1)
    assert_same_weights(got.w, orc.w)


@pytest.mark.parametrize("value_mode", [0, 1])
def test_streamed_long_columns(monkeypatch, value_mode):
    # FAST order, classic layout with chunked long columns (per-batch long arrays streamed too)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "classic")
    monkeypatch.setenv("DLR_LONG_COLUMN", "50")
    D = 2000
    ds = dlr.Dataset.generate(20_000, D, 12, value_mode=value_mode, seed=9, stream=1)
    monkeypatch.setenv("DLR_RESIDENCY", "device")
    ref = run_engine([ds], D, 2, 3000, 0.1, order=dlr.ORDER_FAST)
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_engine([ds], D, 2, 3000, 0.1, order=dlr.ORDER_FAST)
    assert_same_weights(got.w, ref.w)


@pytest.mark.parametrize("mode", [dlr.MODE_SYNC_MEAN, dlr.MODE_ASYNC])
def test_streamed_two_ranks(monkeypatch, mode):
    # world > 1 (loopback group): key-range exchange and, for huge D, the
    # touched exchange, each rank streaming its own shard
    D = 30000
    shards = [dlr.Dataset.generate(2000, D, 20, value_mode=1, seed=4, stream=r + 1) for r in range(2)]
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    got = run_group(shards, D, 2, 512, 0.2, mode=mode)
    orc = oracle.run_worker([_csr(s) for s in shards], D, 2, 512, 0.2, mode=mode)
    assert_same_weights(got.w, orc.w)
    D2 = 1 << 22
    shards = [dlr.Dataset.generate(2000, D2, 10, seed=7, stream=r + 1) for r in range(2)]
    got = run_group(shards, D2, 2, 256, 0.2, mode=mode)
    orc = oracle.run_worker([_csr(s) for s in shards], D2, 2, 256, 0.2, mode=mode)
    assert_same_weights(got.w, orc.w)


def test_streamed_parameter_server_topology(monkeypatch):
    # dlr_worker_gradient / dlr_server_apply on streamed worker shards
    monkeypatch.setenv("DLR_RESIDENCY", "stream")
    D = 123
    shards = [dlr.Dataset.generate(800, D, 14, seed=10, stream=r + 1) for r in range(2)]
    got = run_engine(shards, D, 2, 100, 0.2)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 100, 0.2)
    assert_same_weights(got.w, orc.w)


def test_streamed_residency_reporting_and_limits(monkeypatch):
    D = 5000
    ds = dlr.Dataset.generate(4000, D, 10, seed=2, stream=1)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, 1000)
        assert eng.train_residency() == dlr.RESIDENCY_DEVICE       # auto: fits
        dev_bytes = eng.memory_info()[0]
        eng.set_residency(dlr.RESIDENCY_STREAM)
        nb = eng.load_train(ds, 1000)
        assert eng.train_residency() == dlr.RESIDENCY_STREAM
        assert eng.memory_info()[0] < dev_bytes                     # two batch slots, not the shard
        for b in range(nb):
            eng.train_step(b, 0.1)
        with pytest.raises(dlr.DLRError, match="streamed"):
            eng.stage_time(dlr.STAGE_MARGIN, 0, 2)
        # a band-mode batch (>= 2^21 rows) is one huge step: not streamed per batch
        monkeypatch.setenv("DLR_BAND_ROWS", "16")
        monkeypatch.setenv("DLR_GRAD_KERNEL", "classic")
        with pytest.raises(dlr.DLRError, match="band-mode"):
            eng.load_train(ds, -1)
    finally:
        eng.close()
