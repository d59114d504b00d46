"""The world > 1 engine path on the GPU, against the oracle.

Two transports run the SAME engine code for W ranks (dlr_comm.h):

* the in-process LOOPBACK group (dlr_create_group): W contexts on one
  device, one host thread each -- runs on the 1-GPU box, so every test here
  but the last group executes the key-range all-to-all (rank r receives
  every rank's slice of its key range), the rank-ordered merge + SGD on the
  owned range (k_merge_update), the in-place all-gather at w + r*chunk, the
  touched-list exchange (k_sparse_merge) and the cross-rank load-time
  agreement (batch counts, layout, column order, RankSizes);
* RCCL across processes (bench.py's launcher, one process per GPU): needs
  >= 2 GPUs, skipped otherwise.

Reference: W workers each on its own shard (main.cc:124-170, lr.cc:116-132),
one server applying the merged pushes (main.cc:57-84).  The oracle fixes
the arrival order to rank order (oracle.run_worker), so results are
bitwise."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, ROOT, read_golden_json
from engine_driver import run_engine, run_group
from test_gpu_parity import assert_same_weights, compare_runs, oracle_shard

pytestmark = pytest.mark.gpu

MODES = {"mean": dlr.MODE_SYNC_MEAN, "last": dlr.MODE_SYNC_LAST, "async": dlr.MODE_ASYNC}


def _golden(name):
    meta = read_golden_json("trajectories.json")[name]
    base = os.path.join(GOLDEN, meta["dataset"])
    D = meta["D"]
    shards = [dlr.Dataset.load_libsvm(os.path.join(base, "train", f"part-00{p + 1}"), D)
              for p in range(meta["workers"])]
    test = dlr.Dataset.load_libsvm(os.path.join(base, "test", "part-001"), D)
    return meta, D, shards, test


def _check_golden(res, meta):
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]
    assert [p.astype("<f4").tobytes().hex() for p in res.pulled] == meta["pulled"]
    lines = [f"Iteration {it}, accuracy: {oracle.format_g(oracle.accuracy(c, n))}" for it, c, n, _ in res.tests]
    assert lines == meta["accuracy_lines"]


def test_group_transport_reported():
    engines = dlr.Engine.create_group(100, 3)
    try:
        assert [e.comm_info() for e in engines] == [(3, dlr.TRANSPORT_LOOPBACK)] * 3
    finally:
        for e in engines:
            e.close()
    with dlr.Engine(100) as e:
        assert e.comm_info() == (0, dlr.TRANSPORT_NONE)


GOLDEN_W2 = [n for n, m in read_golden_json("trajectories.json").items() if m["workers"] >= 2]


@pytest.mark.parametrize("layout", ["classic", "lds", "touched"])
@pytest.mark.parametrize("name", GOLDEN_W2)
def test_golden_trajectories_group(monkeypatch, layout, name):
    # frozen oracle trajectories (W = 2, mean / last / async) through the
    # loopback world > 1 step, per gradient layout
    monkeypatch.setenv("DLR_GRAD_KERNEL", layout)
    meta, D, shards, test = _golden(name)
    try:
        res = run_group(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                        test_interval=meta["test_interval"], mode=meta["mode"])
    except dlr.DLRError as e:
        if "do not fit the LDS layout" in str(e):
            pytest.skip("batches too dense for the LDS layout")
        raise
    _check_golden(res, meta)


@pytest.mark.parametrize("name", GOLDEN_W2)
def test_golden_trajectories_group_dense(name):
    meta, D, shards, test = _golden(name)
    res = run_group(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                    test_interval=meta["test_interval"], mode=meta["mode"], dense=True)
    _check_golden(res, meta)


@pytest.fixture(scope="module")
def c1_full():
    D = 123
    shards = [dlr.Dataset.generate(8140, D, 14, seed=10, stream=p + 1, positive_frac=0.24) for p in range(4)]
    test = dlr.Dataset.generate(16281, D, 14, seed=10, stream=100, positive_frac=0.24)
    return D, shards, test


@pytest.mark.parametrize("mode", list(MODES))
def test_c1_local_sh_two_ranks(c1_full, mode):
    # local.sh's topology (2 workers, B = -1, 100 epochs, test every 10)
    D, shards, test = c1_full
    got = run_group(shards[:2], D, 100, -1, 0.2, test=test, test_interval=10, mode=MODES[mode])
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards[:2]], D, 100, -1, 0.2, test=oracle_shard(test, D),
                            test_interval=10, mode=MODES[mode])
    compare_runs(got, orc)


@pytest.mark.parametrize("mode", list(MODES))
def test_four_ranks_minibatch(c1_full, mode):
    D, shards, test = c1_full
    got = run_group(shards, D, 2, 512, 0.2, test=test, test_interval=1, mode=MODES[mode])
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 512, 0.2, test=oracle_shard(test, D),
                            test_interval=1, mode=MODES[mode])
    compare_runs(got, orc)


@pytest.mark.parametrize("W,D", [(3, 7), (4, 5), (5, 3), (2, 1)])
def test_key_ranges_short_and_empty(W, D):
    # ceil(D/W)-sized key ranges with a short or EMPTY last range
    # (dlr_key_range), and ranks that own nothing
    shards = [dlr.Dataset.generate(40, D, min(D, 2), value_mode=1, seed=5, stream=r + 1) for r in range(W)]
    got = run_group(shards, D, 3, 16, 0.3, mode=dlr.MODE_SYNC_MEAN)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 3, 16, 0.3)
    assert_same_weights(got.w, orc.w)


@pytest.mark.parametrize("mode", list(MODES))
def test_touched_exchange_three_ranks(monkeypatch, mode):
    # huge-D touched layout: all-gather of [count | cols | g] blocks, the
    # lowest touching rank merges in rank order (k_sparse_merge)
    D = 1 << 22
    shards = [dlr.Dataset.generate(3000, D, 10, seed=7, stream=r + 1) for r in range(3)]
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(shards[0], 256)
        assert eng.train_layout() == dlr.LAYOUT_TOUCHED
    finally:
        eng.close()
    got = run_group(shards, D, 2, 256, 0.2, mode=MODES[mode])
    orc = oracle.run_worker([_csr(s) for s in shards], D, 2, 256, 0.2, mode=MODES[mode])
    assert_same_weights(got.w, orc.w)


def _c3_shards(W, rows):
    return [dlr.Dataset.generate_hashed(rows, 1 << 24, 39, seed=10, stream=r + 1) for r in range(W)]


def _csr(ds):
    rp, col, val, lab = ds.csr()
    return (rp, col, val), lab


def test_c3_shaped_two_ranks_bands_relabel_bitwise(monkeypatch):
    # C3 structure on 2 ranks: frequency relabeling from the ranks' SUMMED
    # column counts, row bands, the hot-weight margin, key-range exchange of
    # the 2^24 weights; one sequential sum per column (the reference order,
    # default) -> bitwise
    monkeypatch.setenv("DLR_BAND_ROWS", "16384")
    D = 1 << 24
    shards = _c3_shards(2, 70_000)
    got = run_group(shards, D, 2, -1, 0.2)
    orc = oracle.run_worker([_csr(s) for s in shards], D, 2, -1, 0.2)
    assert_same_weights(got.w, orc.w)


def test_c3_shaped_two_ranks_long_phases_within_tolerance(monkeypatch):
    # FAST order: long columns in phases
    monkeypatch.setenv("DLR_BAND_ROWS", "16384")
    D = 1 << 24
    shards = _c3_shards(2, 70_000)
    got = run_group(shards, D, 2, -1, 0.2, order=dlr.ORDER_FAST)
    orc = oracle.run_worker([_csr(s) for s in shards], D, 2, -1, 0.2)
    a, b = got.w.astype(np.float64), orc.w.astype(np.float64)
    assert np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-7)
    one = run_engine(shards, D, 2, -1, 0.2, order=dlr.ORDER_FAST)  # the W = 2 parameter-server topology
    a = one.w.astype(np.float64)
    assert np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-7)


def test_unequal_batch_counts_fail_on_every_rank():
    # a rank with a different batch count must not leave its peers
    # in a collective; every rank fails with the same diagnosis
    D = 50
    shards = [dlr.Dataset.generate(100, D, 5, seed=1, stream=1), dlr.Dataset.generate(300, D, 5, seed=1, stream=2)]
    with pytest.raises(dlr.DLRError, match="different batch counts"):
        run_group(shards, D, 1, 64, 0.1)


def test_rejected_shard_fails_on_every_rank():
    D = 50
    good = dlr.Dataset.generate(100, D, 5, seed=1, stream=1)
    bad = dlr.Dataset.generate(100, D + 1, 5, seed=1, stream=2)  # D mismatch on rank 1
    with pytest.raises(dlr.DLRError, match="D != context D|another rank rejected"):
        run_group([good, bad], D, 1, 64, 0.1)


def test_failed_rank_releases_its_peers():
    # a rank that fails (here: stops before its step) aborts the
    # group; the peer blocked in the step's collective fails at once with
    # the reason instead of waiting for the loopback timeout
    import threading
    import time
    D = 30000
    shards = [dlr.Dataset.generate(1000, D, 20, value_mode=1, seed=3, stream=r + 1) for r in range(2)]
    engines = dlr.Engine.create_group(D, 2)
    err = [None, None]
    try:
        for e, s in zip(engines, shards):
            e.set_weights(dlr.init_weight(D))
        ths = [threading.Thread(target=lambda r=r: engines[r].load_train(shards[r], 100)) for r in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()

        def rank0():
            try:
                engines[0].train_step(0, 0.1)
                engines[0].sync()
            except dlr.DLRError as e:
                err[0] = e

        t0 = time.perf_counter()
        th = threading.Thread(target=rank0)
        th.start()
        time.sleep(0.5)
        engines[1].comm_abort("rank 1 cannot read its shard")
        th.join(timeout=60)
        assert not th.is_alive()
        assert err[0] is not None and "cannot read its shard" in str(err[0])
        assert time.perf_counter() - t0 < 30
        with pytest.raises(dlr.DLRError, match="failed earlier"):
            engines[1].train_step(0, 0.1)
    finally:
        for e in engines:
            e.close()


# ---------------------------------------------------------------- RCCL, one process per GPU


def _visible_gpus() -> int:
    import torch
    return torch.cuda.device_count()


@pytest.mark.parametrize("mode", list(MODES))
def test_rccl_processes_vs_oracle(tmp_path, mode):
    """bench.py's launcher starts one process per GPU (RCCL over xGMI); each
    rank trains its own shard; every rank's final weights must equal the
    oracle's W-worker run bitwise."""
    n = min(_visible_gpus(), 4)
    if n < 2:
        pytest.skip("needs >= 2 GPUs (RCCL refuses two ranks on one device; the loopback tests above cover "
                    "the world > 1 engine path on one GPU)")
    out = tmp_path / "w"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--config", "c1", "--steps", "5",
           "--warmup", "0", "--no-cpu-baseline", "--mode", mode, "--dump-weights", str(out)]
    r = subprocess.run(cmd, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == n and line["exchange"]["rccl_nranks"] == n
    D = 123
    shards = [dlr.Dataset.generate(8140, D, 14, value_mode=0, seed=10, stream=r + 1) for r in range(n)]  # bench.py c1
    steps = 5 + 5  # the un-instrumented and the instrumented pass (no warmup)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, steps, -1, 0.2, mode=MODES[mode])
    for r in range(n):
        w = np.fromfile(f"{out}.rank{r}", dtype=np.float32)
        assert_same_weights(w, orc.w, f"rank {r}")


@pytest.mark.parametrize("layout", ["lds", "classic", "touched"])
@pytest.mark.parametrize("B", [7, 1001, -1])
def test_sparse_layouts_two_ranks_valued(monkeypatch, layout, B):
    # a sparse valued shard that fits the LDS layout (the golden C1 shards
    # are too dense for it), per layout, wrapping batches included
    monkeypatch.setenv("DLR_GRAD_KERNEL", layout)
    D = 30000  # sparse enough for the LDS layout's <= 255 entries per 64-column block and phase
    shards = [dlr.Dataset.generate(1000, D, 20, value_mode=1, seed=3, stream=r + 1) for r in range(2)]
    got = run_group(shards, D, 2, B, 0.1, mode=dlr.MODE_SYNC_MEAN)
    orc = oracle.run_worker([_csr(s) for s in shards], D, 2, B, 0.1)
    compare_runs(got, orc)


def test_rank_failing_mid_load_releases_its_peers(monkeypatch):
    # a rank that fails AFTER the load agreement (here: DLR_PM=1
    # and its rows are too long for the product margin) must not leave its
    # peer blocked in the load's later collectives: it aborts the group
    # (run_group's error path), and the peer's load fails with the reason
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    import time
    D = 300_000
    ok = dlr.Dataset.generate(1200, D, 18, value_mode=1, seed=13, stream=1)
    too_long = dlr.Dataset.generate(1200, D, 200, value_mode=1, seed=13, stream=2)  # > 128 entries a row
    t0 = time.perf_counter()
    with pytest.raises(dlr.DLRError):
        run_group([ok, too_long], D, 1, 300, 0.2)
    assert time.perf_counter() - t0 < 120, "the peer waited for the loopback timeout"
