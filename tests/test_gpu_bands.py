"""Row bands (dlr_train_band_rows): for large batches the classic layout's
short columns are summed band by band -- one launch per band of 2^k batch
rows, each column's running sum continued from band to band in batch-row
order (dlr_kernels.hip "Row-band layout").  That is lr.cc:35-39's sequential
order, so results must be bitwise those of the single-pass classic kernel
and of the oracle.  DLR_BAND_ROWS forces small bands so the golden C1
trajectories and reduced C3-shaped shards exercise many bands, ragged last
bands, empty bands, both row widths (uint16 for <= 65,536-row batches, else
uint32), unit and fp32 values, the pushed gradient (N > 1 path) and the
key-range exchange.  Under the FAST summation order (opt-in,
dlr_set_summation_order) long columns in band mode are summed per row phase
(deterministic, within the 1e-5*|b| + 1e-7 bar); in the reference order
(default) every column is one chain across the bands."""
from __future__ import annotations

import os

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, read_golden_json
from engine_driver import run_engine
from test_gpu_layouts import _c3_shards, _csr_shard
from test_gpu_parity import assert_same_weights, compare_runs, oracle_shard

# band mode's FAST long-column threshold (dlr_engine.cpp, DLR_LONG_COLUMN):
# under ORDER_FAST columns with more entries than this are summed in phases /
# pieces
BAND_LONG_COLUMN = 2048

pytestmark = pytest.mark.gpu


@pytest.fixture
def classic(monkeypatch):
    monkeypatch.setenv("DLR_GRAD_KERNEL", "classic")


def _band_rows(ds, D, B, order=dlr.ORDER_REFERENCE):
    eng = dlr.Engine(D)
    try:
        eng.set_summation_order(order)
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, B)
        assert eng.train_layout() == dlr.LAYOUT_CLASSIC
        return eng.train_band_rows()
    finally:
        eng.close()


@pytest.mark.parametrize("rows", [2, 16, 1024])
@pytest.mark.parametrize("name", ["c1_W1_Bfull_mean", "c1_W1_B7_mean", "c1_W2_B64_async", "real_W2_B50_mean"])
def test_golden_trajectories_banded(classic, monkeypatch, rows, name):
    monkeypatch.setenv("DLR_BAND_ROWS", str(rows))
    meta = read_golden_json("trajectories.json")[name]
    base = os.path.join(GOLDEN, meta["dataset"])
    D = meta["D"]
    shards = [dlr.Dataset.load_libsvm(os.path.join(base, "train", f"part-00{p + 1}"), D)
              for p in range(meta["workers"])]
    B = meta["batch_size"] if meta["batch_size"] > 0 else shards[0].n_rows
    if B <= rows:
        pytest.skip("batch not larger than one band: no bands")
    assert _band_rows(shards[0], D, meta["batch_size"]) == rows
    test = dlr.Dataset.load_libsvm(os.path.join(base, "test", "part-001"), D)
    res = run_engine(shards, D, meta["num_iteration"], meta["batch_size"], meta["learning_rate"], test=test,
                     test_interval=meta["test_interval"], mode=meta["mode"])
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]
    assert [p.astype("<f4").tobytes().hex() for p in res.pulled] == meta["pulled"]


def test_band_rows_choice(classic, monkeypatch):
    ds = dlr.Dataset.generate(3000, 5000, 10, seed=2, stream=1)
    monkeypatch.delenv("DLR_BAND_ROWS", raising=False)
    assert _band_rows(ds, 5000, -1) == 0            # default bands start at 2^21-row batches
    monkeypatch.setenv("DLR_BAND_ROWS", "1000")      # rounded down to a power of two
    assert _band_rows(ds, 5000, -1) == 512
    assert _band_rows(ds, 5000, 512) == 0           # one band: no bands
    monkeypatch.setenv("DLR_BAND_ROWS", "0")
    assert _band_rows(ds, 5000, -1) == 0


@pytest.mark.parametrize("B", [7, 1001, 2500, -1])
@pytest.mark.parametrize("value_mode", [0, 1])
def test_batch_sizes_banded(classic, monkeypatch, B, value_mode):
    # wrapping batches, a batch larger than the shard, ragged last bands
    monkeypatch.setenv("DLR_BAND_ROWS", "4")
    D = 3000
    ds = dlr.Dataset.generate(1000, D, 20, value_mode=value_mode, seed=3, stream=1)
    eng = run_engine([ds], D, 2, B, 0.1)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 2, B, 0.1)
    compare_runs(eng, orc)


def test_ragged_and_empty_bands(classic, monkeypatch):
    # rows with no entries make whole bands empty (a band with no pairs)
    monkeypatch.setenv("DLR_BAND_ROWS", "8")
    rng = np.random.default_rng(5)
    D, n = 4000, 1200
    lens = rng.integers(0, 30, size=n)
    lens[100:180] = 0      # 80 empty rows: >= 9 empty bands of 8
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(D, k, replace=False)) for k in lens]).astype(np.int32)
    val = rng.integers(1, 10001, size=len(col)).astype(np.float32) / np.float32(10000)
    lab = rng.integers(0, 2, size=n).astype(np.int32)
    ds = dlr.Dataset.from_csr(rp, col, val, lab, D)
    eng = run_engine([ds], D, 2, 600, 0.3)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 2, 600, 0.3)
    compare_runs(eng, orc)


@pytest.mark.parametrize("rows", [4096, 32768])
def test_c3_bands_bitwise_without_chunking(monkeypatch, rows):
    # the reference order (default): every column one sequential sum,
    # carried across bands -- bitwise the oracle (uint32 rows: the
    # full-shard batch has > 65,536 rows); a stray DLR_LONG_COLUMN does not
    # change the order
    monkeypatch.setenv("DLR_LONG_COLUMN", "50")
    monkeypatch.setenv("DLR_BAND_ROWS", str(rows))
    D = 1 << 24
    shards = _c3_shards(1, rows=80_000)
    assert _band_rows(shards[0], D, -1) == rows
    eng = run_engine(shards, D, 2, -1, 0.2)
    assert not eng_fast(shards[0], D)
    orc = oracle.run_worker([_csr_shard(s) for s in shards], D, 2, -1, 0.2)
    compare_runs(eng, orc)


def eng_fast(ds, D):
    """The loaded shard's reported order is FAST (dlr_summation_order)."""
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, -1)
        return eng.summation_order() == dlr.ORDER_FAST
    finally:
        eng.close()


def _within(a, b, rel=1e-5, floor=1e-7):
    a, b = a.astype(np.float64), b.astype(np.float64)
    err = np.abs(a - b) - (rel * np.abs(b) + floor)
    assert err.max() <= 0, f"max excess {err.max():.3g}"


@pytest.mark.parametrize("W", [1, 2])
def test_c3_bands_long_phases_within_tolerance(monkeypatch, W):
    # band mode: long columns summed per row phase (16,384 rows) and the
    # phase partials combined by a fixed tree -- deterministic, within the
    # north-star bar of the reference's single sequential sum
    D = 1 << 24
    shards = _c3_shards(W, rows=80_000)
    monkeypatch.setenv("DLR_BAND_ROWS", "8192")
    assert _band_rows(shards[0], D, -1, dlr.ORDER_FAST) == 8192
    got = run_engine(shards, D, 3, -1, 0.2, order=dlr.ORDER_FAST)
    orc = oracle.run_worker([_csr_shard(s) for s in shards], D, 3, -1, 0.2)
    _within(got.w, orc.w)
    again = run_engine(shards, D, 3, -1, 0.2, order=dlr.ORDER_FAST)
    assert_same_weights(again.w, got.w)


@pytest.mark.parametrize("order", [dlr.ORDER_REFERENCE, dlr.ORDER_FAST])
@pytest.mark.parametrize("W", [1, 2])
def test_band_pipeline_bitwise_vs_sequential(monkeypatch, W, order):
    # band mode runs the margin band by band with each band's gradient on a
    # second stream beside the next band's margin, the long-column phases
    # (FAST) after the last margin (DLR_BAND_PIPE=0: margin, then gradient):
    # the same kernels on the same data -- bitwise the same weights
    D = 1 << 24
    shards = _c3_shards(W, rows=80_000)
    monkeypatch.setenv("DLR_BAND_ROWS", "8192")
    got = run_engine(shards, D, 3, -1, 0.2, order=order)
    monkeypatch.setenv("DLR_BAND_PIPE", "0")
    ref = run_engine(shards, D, 3, -1, 0.2, order=order)
    assert_same_weights(got.w, ref.w)


@pytest.mark.parametrize("hot", ["64", "2000", "0"])
@pytest.mark.parametrize("W", [1, 2])
def test_band_hot_pairs_bitwise(monkeypatch, W, hot):
    # REFERENCE order, band mode, pipelined: the hot columns' pairs (>= hot
    # entries in the batch; DLR_BAND_HOT, "0" = none) run in k_band_hot on
    # a third stream, band after band, the other columns in k_grad_band
    # beside them -- the same chains: bitwise the oracle (and the sequential
    # DLR_BAND_PIPE=0 path, which keeps every pair in k_grad_band)
    D = 1 << 24
    shards = _c3_shards(W, rows=80_000)
    monkeypatch.setenv("DLR_BAND_ROWS", "8192")
    monkeypatch.setenv("DLR_BAND_HOT", hot)
    got = run_engine(shards, D, 3, -1, 0.2)
    orc = oracle.run_worker([_csr_shard(s) for s in shards], D, 3, -1, 0.2)
    compare_runs(got, orc)
    monkeypatch.setenv("DLR_BAND_PIPE", "0")
    seq = run_engine(shards, D, 3, -1, 0.2)
    assert_same_weights(got.w, seq.w)


@pytest.mark.parametrize("value_mode", [1, 2])
def test_band_hot_pairs_valued(classic, monkeypatch, value_mode):
    # fp32 values (the hot kernel's products r * x, uint16 rows at this
    # size): bitwise the oracle with every column of >= 32 entries hot
    monkeypatch.setenv("DLR_BAND_ROWS", "16")
    monkeypatch.setenv("DLR_BAND_HOT", "32")
    D = 400
    ds = dlr.Dataset.generate(700, D, 40, value_mode=value_mode, seed=37, stream=3)
    eng = run_engine([ds], D, 2, -1, 0.3)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 2, -1, 0.3)
    compare_runs(eng, orc)


def test_c3_banded_pushed_gradient(monkeypatch):
    # the N > 1 path's pushed gradient (non-fused finalize), FAST order:
    # short columns bitwise the unbanded classic kernel's, long columns
    # within 1e-5 of the oracle's sequential sums
    D = 1 << 24
    ds = _c3_shards(1, rows=60_000)[0]
    rp, col, val, lab = ds.csr()
    hot = np.bincount(col, minlength=D) > BAND_LONG_COLUMN
    assert hot.sum() >= 30
    w0 = dlr.init_weight(D)
    out = {}
    for rows in ("0", "4096"):
        monkeypatch.setenv("DLR_BAND_ROWS", rows)
        eng = dlr.Engine(D)
        try:
            eng.set_summation_order(dlr.ORDER_FAST)
            eng.set_weights(w0)
            eng.load_train(ds, -1)
            assert eng.train_band_rows() == int(rows)
            out[rows] = eng.worker_gradient(0, 1.0)
        finally:
            eng.close()
    assert_same_weights(out["4096"][~hot], out["0"][~hot], "short-column gradient")
    go = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(len(lab), -1, 0), w0)
    a, b = out["4096"][hot].astype(np.float64), go[hot].astype(np.float64)
    assert np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-9), np.max(np.abs(a - b) / np.abs(b))


@pytest.mark.parametrize("B", [2000, 3000, -1])
@pytest.mark.parametrize("value_mode", [0, 1])
def test_long_phases_small_threshold(classic, monkeypatch, B, value_mode):
    # many long columns (threshold 50 entries), several batches each with its
    # own phases (row16 batches; B = 3,000 wraps to row 0), valued and unit
    # shards: within tolerance of the oracle and deterministic
    monkeypatch.setenv("DLR_BAND_ROWS", "256")
    monkeypatch.setenv("DLR_LONG_COLUMN", "50")
    D = 2000
    ds = dlr.Dataset.generate(20_000, D, 12, value_mode=value_mode, seed=9, stream=1)
    got = run_engine([ds], D, 2, B, 0.1, order=dlr.ORDER_FAST)
    orc = oracle.run_worker([_csr_shard(ds)], D, 2, B, 0.1)
    _within(got.w, orc.w)
    again = run_engine([ds], D, 2, B, 0.1, order=dlr.ORDER_FAST)
    assert_same_weights(again.w, got.w)


def test_banded_forced_collectives(classic, monkeypatch):
    # key-range all-to-all + merge + all-gather (1-rank communicator)
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    monkeypatch.setenv("DLR_BAND_ROWS", "16")
    meta = read_golden_json("trajectories.json")["c1_W1_Bfull_mean"]
    base = os.path.join(GOLDEN, meta["dataset"])
    ds = dlr.Dataset.load_libsvm(os.path.join(base, "train", "part-001"), 123)
    res = run_engine([ds], 123, meta["num_iteration"], meta["batch_size"], meta["learning_rate"],
                     mode=meta["mode"])
    assert res.w.astype("<f4").tobytes().hex() == meta["w"]


def _long_phase_order(prods_by_col, piece, Bn, w, C_=1.0, phase=16384):
    """The documented long-column order in band mode (dlr_kernels.hip
    k_long_phase + k_long_combine): per column, its products in
    batch-row order cut at 16,384-row phase boundaries, each phase's run cut
    into pieces of `piece` entries summed sequentially in fp32 from +0; the
    piece partials (phase by phase) added by 64 lanes -- lane l takes partials
    l, l + 64, ... in order -- and the lane sums by the xor-butterfly tree
    (off 32, 16, ..., 1; lane 0's value); then lr.cc:40."""
    out = {}
    f32 = np.float32
    for j, (pos, prod) in prods_by_col.items():
        parts = []
        ph = pos // phase
        for p in np.unique(ph):
            run = prod[ph == p]
            for o in range(0, len(run), piece):
                parts.append(np.cumsum(run[o:o + piece], dtype=f32)[-1])
        parts = np.asarray(parts, dtype=f32)
        v = np.zeros(64, dtype=f32)
        for l in range(64):
            if len(parts[l::64]):
                v[l] = np.cumsum(parts[l::64], dtype=f32)[-1]
        for off in (32, 16, 8, 4, 2, 1):
            v = (v + v[np.arange(64) ^ off]).astype(f32)
        G = v[0]
        l2 = f32(f32(f32(C_) * w[j]) / f32(Bn))
        out[j] = f32(np.float64(G) / np.float64(Bn) + np.float64(l2))
    return out


@pytest.mark.parametrize("piece", [63, 64, 7, 1024])
def test_long_phase_order_bitwise(monkeypatch, piece):
    # pins k_long_phase / k_long_combine to their documented summation order
    # bit for bit (a restatement in numpy on the oracle's residuals), across
    # piece sizes: 63 (default), 64, short pieces (7: many pieces per lane)
    # and 1,024-entry pieces (tasks whose entries span two windows)
    monkeypatch.setenv("DLR_BAND_ROWS", "8192")
    monkeypatch.setenv("DLR_LONG_PIECE", str(piece))
    D = 1 << 24
    ds = _c3_shards(1, rows=60_000)[0]
    rp, col, val, lab = ds.csr()
    N = len(lab)
    counts = np.bincount(col, minlength=D)
    long_cols = np.flatnonzero(counts > BAND_LONG_COLUMN)
    assert len(long_cols) >= 30
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_summation_order(dlr.ORDER_FAST)
        eng.set_weights(w0)
        eng.load_train(ds, -1)
        assert eng.train_band_rows() == 8192 and eng.summation_order() == dlr.ORDER_FAST
        got = eng.worker_gradient(0, 1.0)
    finally:
        eng.close()
    rows = oracle.batch_rows(N, -1, 0)
    g_orc, resid = oracle.grad_csr((rp, col, val), lab, rows, w0, return_resid=True)
    row_of = np.repeat(np.arange(N), np.diff(rp))
    prods = {}
    for j in long_cols:
        k = np.flatnonzero(col == j)                 # entries of column j, rows ascending
        pos = row_of[k]
        prods[j] = (pos, (resid[pos] * val[k]).astype(np.float32))
    want = _long_phase_order(prods, piece, N, w0)
    bad = [j for j in long_cols if np.float32(got[j]).tobytes() != want[j].tobytes()]
    assert not bad, f"{len(bad)} long columns off the documented order, e.g. {bad[:3]}"
    # and the short columns stay the reference's sequential sums
    short = counts <= BAND_LONG_COLUMN
    assert_same_weights(got[short], g_orc[short], "short-column gradient")



def _hot_stream_run(ds, D, steps, hot, stream, band_rows="8192", counters=None, extra_env=None):
    import os as _os
    env = {"DLR_BAND_ROWS": band_rows, "DLR_BAND_HOT": hot, "DLR_HOT_STREAM": stream, "DLR_GRAD_KERNEL": "classic"}
    env.update(extra_env or {})
    old = {k: _os.environ.get(k) for k in env}
    _os.environ.update(env)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, -1)
        nh = eng.train_hot_columns()
        for _ in range(steps):
            eng.train_step(0, 0.2, 1.0)
        w = eng.get_weights()
        if counters is not None:
            counters.update(eng.stage_counters())
        return w, nh
    finally:
        eng.close()
        for k, v in old.items():
            if v is None:
                _os.environ.pop(k, None)
            else:
                _os.environ[k] = v


@pytest.mark.parametrize("hot", ["2000", "6000"])
def test_hot_stream_bitwise(hot):
    # the hot columns' chains from the product stream (the margin writes
    # fl32(r_i * x_ij) of each hot entry, ONE k_hot_chain launch adds every
    # hot column over all bands, band s once its flag is up): bitwise the
    # per-band k_band_hot chains (DLR_HOT_STREAM=0) and the oracle
    D = 1 << 24
    ds = _c3_shards(1, rows=80_000)[0]
    got, nh = _hot_stream_run(ds, D, 3, hot, "1")
    assert 0 < nh <= 128, nh
    ref, nh0 = _hot_stream_run(ds, D, 3, hot, "0")
    assert nh0 == 0
    assert_same_weights(got, ref, "hot stream vs k_band_hot")
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    for _ in range(3):
        g = oracle.grad_csr((rp, col, val), lab, np.arange(len(lab)), w)
        oracle.server_update(w, [g], 0.2)
    assert_same_weights(got, w, "hot stream vs oracle")


def test_hot_stream_valued_and_ragged_bands():
    # fp32 values (the products r * x in the margin) and a last band of a
    # few rows; bands of 4,096 rows so columns hold segments in many bands
    D = 1 << 20
    rng = np.random.default_rng(5)
    n = 30_001
    hot_cols = np.array([3, 17, 40000], dtype=np.int64)
    rows, cols = [], []
    for i in range(n):
        c = set(rng.choice(D, 12, replace=False).tolist())
        for h in hot_cols:
            if rng.random() < 0.3:
                c.add(int(h))
        c = sorted(c)
        rows.append(len(c))
        cols.extend(c)
    rp = np.concatenate([[0], np.cumsum(rows)]).astype(np.int64)
    col = np.asarray(cols, dtype=np.int32)
    val = rng.integers(1, 10001, size=len(col)).astype(np.float32) / np.float32(10000)
    lab = rng.integers(0, 2, size=n).astype(np.int32)
    ds = dlr.Dataset.from_csr(rp, col, val, lab, D)
    import os as _os
    _os.environ["DLR_MARGIN_HOT"] = "1"
    try:
        got, nh = _hot_stream_run(ds, D, 2, "5000", "1", band_rows="4096")
        ref, _ = _hot_stream_run(ds, D, 2, "5000", "0", band_rows="4096")
    finally:
        _os.environ.pop("DLR_MARGIN_HOT", None)
    assert nh == 3, nh
    assert_same_weights(got, ref, "hot stream vs k_band_hot (valued)")
    w = dlr.init_weight(D)
    for _ in range(2):
        g = oracle.grad_csr((rp, col, val), lab, np.arange(n), w)
        oracle.server_update(w, [g], 0.2)
    assert_same_weights(got, w, "hot stream vs oracle (valued)")


def _chain_launches(nbands):
    # k_hot_chain launches per step: one after the margins of band 2 (the
    # first two bands'), one after the last margin, and the final one the
    # stream orders after the last margin (DevHotChain)
    return (1 if nbands <= 2 else 2) + 1


def test_hot_stream_serialised_kernels_no_giveup(tmp_path):
    # every chain launch is queued after the margins of its last band, so
    # even with every kernel serialised (AMD_SERIALIZE_KERNEL=3, as under
    # counter collection) no launch waits for a flag: zero give-ups, the
    # same bits as the concurrent run
    import json
    import subprocess
    import sys
    D = 1 << 24
    ds = _c3_shards(1, rows=80_000)[0]
    cnt = {}
    got, nh = _hot_stream_run(ds, D, 2, "2000", "1", counters=cnt)
    assert nh > 0
    nbands = -(-80_000 // 8192)
    assert cnt["hot_chain_launches"] == 2 * _chain_launches(nbands), cnt
    assert cnt["hot_giveups"] == 0, cnt
    out = tmp_path / "w.npy"
    cout = tmp_path / "c.json"
    code = (
        "import sys, json, numpy as np\n"
        "sys.path.insert(0, %r); sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import test_gpu_bands as t, distlr_amd as dlr\n"
        "ds = t._c3_shards(1, rows=80_000)[0]\n"
        "cnt = {}\n"
        "w, nh = t._hot_stream_run(ds, 1 << 24, 2, '2000', '1', counters=cnt)\n"
        "assert nh > 0\n"
        "np.save(%r, w)\n"
        "json.dump(cnt, open(%r, 'w'))\n"
    ) % (os.path.dirname(os.path.abspath(__file__)), os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "dist-lr_amd"), os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "oracle"), str(out), str(cout))
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
    assert_same_weights(np.load(out), got, "serialised kernels vs concurrent")
    scnt = json.load(open(cout))
    assert scnt["hot_giveups"] == 0, scnt


def test_hot_stream_with_collective_streams_no_giveup():
    # the C3 shape's hot chains with the world > 1 stream
    # set on one GPU -- RCCL (one rank: DLR_FORCE_COLLECTIVES=1) adds its
    # streams and the exchange stream beside the engine's three -- zero
    # give-ups and the oracle's bits
    D = 1 << 24
    ds = _c3_shards(1, rows=80_000)[0]
    cnt = {}
    got, nh = _hot_stream_run(ds, D, 3, "2000", "1", counters=cnt, extra_env={"DLR_FORCE_COLLECTIVES": "1"})
    assert nh > 0
    assert cnt["hot_giveups"] == 0, cnt
    assert cnt["hot_chain_launches"] == 3 * _chain_launches(-(-80_000 // 8192)), cnt
    (rp, col, val), lab = _csr_shard(ds)
    w = dlr.init_weight(D)
    for _ in range(3):
        g = oracle.grad_csr((rp, col, val), lab, np.arange(80_000), w)
        oracle.server_update(w, [g], 0.2)
    assert_same_weights(got, w, "hot stream under collectives vs oracle")
