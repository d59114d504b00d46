"""GPU parity: the HIP path (through the C-ABI) against the oracle on the
same inputs.  Bar (BASELINE.json north_star): weights within 1e-5 relative;
the kernels keep the reference's summation order, so we assert BITWISE
equality of weights and pulled snapshots, equal correct counts (hence equal
accuracy lines), and log-loss within 1e-9 relative (our metric; the oracle
sums it in another order with glibc instead of OCML transcendental)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, read_golden_json
from engine_driver import run_engine
from parse_format import csr_to_dense

pytestmark = pytest.mark.gpu

LL_RTOL = 1e-9


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def assert_same_weights(got, want, what="w"):
    g, w = bits(got), bits(want)
    if not np.array_equal(g, w):
        diff = np.nonzero(g != w)[0]
        a = np.asarray(got, np.float64)[diff]
        b = np.asarray(want, np.float64)[diff]
        rel = np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30))
        raise AssertionError(f"{what}: {len(diff)} of {len(g)} weights differ (first {diff[:5]}, max rel {rel:.3g})")


def oracle_shard(ds: dlr.Dataset, D: int):
    rp, col, val, lab = ds.csr()
    return csr_to_dense(rp, col, val, D), lab


def compare_runs(eng, orc):
    assert_same_weights(eng.w, orc.w)
    for r, (a, b) in enumerate(zip(eng.pulled, orc.pulled)):
        assert_same_weights(a, b, f"pulled[{r}]")
    assert len(eng.tests) == len(orc.tests)
    for (it, c, n, ll), (it2, c2, n2, ll2) in zip(eng.tests, orc.tests):
        assert (it, c, n) == (it2, c2, n2)
        assert abs(ll - ll2) <= LL_RTOL * abs(ll2)


@pytest.mark.parametrize("name", list(read_golden_json("trajectories.json").keys()))
def test_golden_trajectories(name):
    meta = read_golden_json("trajectories.json")[name]
    base = os.path.join(GOLDEN, meta["dataset"])
    D = meta["D"]
    shards = [dlr.Dataset.load_libsvm(os.path.join(base, "train", f"part-00{p + 1}"), D)
              for p in range(meta["workers"])]
    test = dlr.Dataset.load_libsvm(os.path.join(base, "test", "part-001"), D)
    res = run_engine(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                     test_interval=meta["test_interval"], mode=meta["mode"])
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]
    assert [p.astype("<f4").tobytes().hex() for p in res.pulled] == meta["pulled"]
    lines = [f"Iteration {it}, accuracy: {oracle.format_g(oracle.accuracy(c, n))}" for it, c, n, _ in res.tests]
    assert lines == meta["accuracy_lines"]
    for (_, _, _, ll), t in zip(res.tests, meta["tests"]):
        assert abs(ll - t[3]) <= LL_RTOL * abs(t[3])
    assert dlr.format_model(res.pulled[0]) == meta["model_rank0"]


@pytest.fixture(scope="module")
def c1_full():
    """C1 (local.sh topology): D=123, 4 shards x 8140 rows, 16,281 test rows."""
    D = 123
    shards = [dlr.Dataset.generate(8140, D, 14, seed=10, stream=p + 1, positive_frac=0.24) for p in range(4)]
    test = dlr.Dataset.generate(16281, D, 14, seed=10, stream=100, positive_frac=0.24)
    return D, shards, test


def test_c1_full_local_sh_one_worker(c1_full):
    D, shards, test = c1_full
    eng = run_engine(shards[:1], D, 100, -1, 0.2, test=test, test_interval=10)
    orc = oracle.run_worker([oracle_shard(shards[0], D)], D, 100, -1, 0.2, test=oracle_shard(test, D),
                            test_interval=10)
    compare_runs(eng, orc)


@pytest.mark.parametrize("mode", [dlr.MODE_SYNC_MEAN, dlr.MODE_SYNC_LAST])
def test_c1_full_local_sh_two_workers(c1_full, mode):
    D, shards, test = c1_full
    eng = run_engine(shards[:2], D, 100, -1, 0.2, test=test, test_interval=10, mode=mode)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards[:2]], D, 100, -1, 0.2, test=oracle_shard(test, D),
                            test_interval=10, mode=mode)
    compare_runs(eng, orc)


def test_c1_four_workers_async_minibatch(c1_full):
    D, shards, test = c1_full
    eng = run_engine(shards, D, 2, 512, 0.2, test=test, test_interval=1, mode=dlr.MODE_ASYNC)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 512, 0.2, test=oracle_shard(test, D),
                            test_interval=1, mode=dlr.MODE_ASYNC)
    compare_runs(eng, orc)


@pytest.mark.parametrize("B", [1, 7, 100, 999, 1000, 1001, 2500, -1])
def test_batch_sizes_and_wraps(B):
    # B=1000 divides N; others wrap at the epoch end; 2500 > N wraps twice.
    D = 300
    ds = dlr.Dataset.generate(1000, D, 20, value_mode=1, seed=3, stream=1)
    eng = run_engine([ds], D, 2, B, 0.1)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 2, B, 0.1)
    compare_runs(eng, orc)


def test_uint32_row_index_path():
    # B > 65536: the column-major copy stores 32-bit batch rows.
    D = 5000
    ds = dlr.Dataset.generate(70000, D, 8, value_mode=1, seed=4, stream=1)
    eng = run_engine([ds], D, 2, -1, 0.5)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 2, -1, 0.5)
    compare_runs(eng, orc)


def test_long_rows_span_many_windows():
    # rows of 2,900 entries: a wave's rows span many LDS windows.
    D = 3000
    ds = dlr.Dataset.generate(200, D, 2900, value_mode=1, seed=5, stream=1)
    test = dlr.Dataset.generate(130, D, 2900, value_mode=1, seed=5, stream=2)
    eng = run_engine([ds], D, 3, 64, 0.01, test=test, test_interval=1)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 3, 64, 0.01, test=oracle_shard(test, D), test_interval=1)
    compare_runs(eng, orc)


def test_ragged_and_empty_rows():
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
    test = dlr.Dataset.from_csr(rp, col, val, 1 - lab, D)
    eng = run_engine([ds], D, 3, 257, 0.3, test=test, test_interval=1)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 3, 257, 0.3, test=oracle_shard(test, D), test_interval=1)
    compare_runs(eng, orc)


def test_single_feature_and_single_row():
    ds = dlr.Dataset.from_csr([0, 1], [0], [1.0], [1], 1)
    eng = run_engine([ds], 1, 5, -1, 0.2)
    orc = oracle.run_worker([oracle_shard(ds, 1)], 1, 5, -1, 0.2)
    compare_runs(eng, orc)


def test_c2_shaped_steps():
    # The headline kernel shape: D = 1M features, 50 nnz/row, B = 65,536
    # (rows reduced to 200k so the oracle finishes in seconds).
    D = 1_000_000
    ds = dlr.Dataset.generate(200_000, D, 50, value_mode=1, seed=10, stream=1)
    rp, col, val, lab = ds.csr()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        nb = eng.load_train(ds, 65536)
        assert nb == 4
        w = w0.copy()
        for b in range(nb + 1):          # one epoch + the first batch of the next
            bb = b % nb
            eng.train_step(bb, 0.2, 1.0)
            g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(len(lab), 65536, bb), w)
            oracle.server_update(w, [g], 0.2)
        assert_same_weights(eng.get_weights(), w)
    finally:
        eng.close()


def test_forced_collectives_path(monkeypatch):
    # The RCCL exchange (all-to-all + merge kernel + all-gather) with a
    # 1-rank communicator must equal the fused single-rank step.
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    meta = read_golden_json("trajectories.json")["c1_W1_B7_mean"]
    base = os.path.join(GOLDEN, meta["dataset"])
    ds = dlr.Dataset.load_libsvm(os.path.join(base, "train", "part-001"), 123)
    test = dlr.Dataset.load_libsvm(os.path.join(base, "test", "part-001"), 123)
    res = run_engine([ds], 123, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                     test_interval=meta["test_interval"], mode=meta["mode"])
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]


def test_predict_counts_and_logloss():
    D = 2000
    ds = dlr.Dataset.generate(5000, D, 30, value_mode=1, seed=8, stream=1)
    test = dlr.Dataset.generate(33333, D, 30, value_mode=1, seed=8, stream=2)
    eng = dlr.Engine(D)
    try:
        w = (dlr.init_weight(D) - np.float32(0.5)).astype(np.float32)
        eng.set_weights(w)
        eng.load_test(test)
        c, n, ll = eng.predict()
        c2, ll2 = oracle.predict_csr(test.csr()[:3], test.csr()[3], w)
        assert (c, n) == (c2, 33333)
        assert abs(ll - ll2) <= LL_RTOL * abs(ll2)
    finally:
        eng.close()


def test_errors_are_loud():
    eng = dlr.Engine(10)
    try:
        with pytest.raises(dlr.DLRError):
            eng.train_step(0, 0.1)                      # nothing loaded
        with pytest.raises(dlr.DLRError):
            eng.set_weights(np.zeros(9, np.float32))     # wrong D
        ds = dlr.Dataset.generate(10, 11, 3)
        with pytest.raises(dlr.DLRError):
            eng.load_train(ds, 4)                       # D mismatch
    finally:
        eng.close()


def _skewed_a9a_shard(seed, n=8140, D=123, k=14):
    """a9a-like skew: a few columns (sex, race, native-country, capital-gain
    bins...) appear in most rows -- >4,096 entries each in an 8,140-row
    full-shard batch -- the rest fill each row up to k columns."""
    rng = np.random.default_rng(seed)
    hot = np.array([2, 9, 37, 60, 71, 95, 110, 119])
    p_hot = np.array([0.92, 0.85, 0.67, 0.6, 0.55, 0.51, 0.8, 0.7])
    rows = []
    for _ in range(n):
        cols = set(hot[rng.random(len(hot)) < p_hot].tolist())
        while len(cols) < k:
            cols.add(int(rng.integers(0, D)))
        rows.append(sorted(cols))
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    col = np.concatenate(rows).astype(np.int32)
    val = np.ones(len(col), np.float32)
    lab = (rng.random(n) < 0.24).astype(np.int32)
    return dlr.Dataset.from_csr(rp, col, val, lab, D)


@pytest.mark.parametrize("W", [1, 2])
def test_skewed_a9a_full_shard_bitwise(W):
    # local.sh's shape (B = -1 over 8,140 rows) with columns in
    # more than half of the rows must stay bitwise (no chunked long-column
    # sums outside band mode)
    D = 123
    shards = [_skewed_a9a_shard(40 + r) for r in range(W)]
    assert int(np.bincount(shards[0].csr()[1], minlength=D).max()) > 4096
    eng = run_engine(shards, D, 100, -1, 0.2)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 100, -1, 0.2)
    compare_runs(eng, orc)
