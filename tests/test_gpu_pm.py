"""Product margin (dlr_kernels.hip "Product margin", dlr_train_product_margin):
the margin of lr.cc:108-114 formed as products by column slice (pass 1, from
LDS-staged weights; fused into the previous step's gradient on one rank) and
row sums from LDS (pass 2).  Same products, same column order of additions
from +0, so every result must be BITWISE the gather margin's -- and the
oracle's -- whether pass 1 ran fused (the next batch guessed right), on its
own (a guess missed, the weights changed in between, world > 1), or not at
all (DLR_PM=0)."""
from __future__ import annotations

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from engine_driver import run_engine, run_group
from test_gpu_parity import assert_same_weights, compare_runs, oracle_shard

pytestmark = pytest.mark.gpu


def _ragged(seed, D, n, max_len=100, empty=300):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, size=n)
    lens[rng.choice(n, empty, replace=False)] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(D, k, replace=False)) for k in lens]).astype(np.int32)
    val = rng.integers(1, 10001, size=len(col)).astype(np.float32) / np.float32(10000)
    lab = rng.integers(0, 2, size=n).astype(np.int32)
    return dlr.Dataset.from_csr(rp, col, val, lab, D)


# Shapes: a (64-row block, 4,096-column slice) chunk holds <= 256 products,
# so D >= ~1,024 x nnz per row here.


def _mode_of(ds, D, B):
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, B)
        return eng.train_product_margin()
    finally:
        eng.close()


def _rounds_of(ds, D, B):
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, B)
        return eng.train_row_rounds()
    finally:
        eng.close()


@pytest.fixture(params=["fused-mg", "fused", "separate"])
def pm_on(request, monkeypatch):
    # fused-mg: pass 2 in the gradient's launch too (DLR_PM_MG, the default)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    monkeypatch.setenv("DLR_PM_FUSED", "0" if request.param == "separate" else "1")
    monkeypatch.setenv("DLR_PM_MG", "1" if request.param == "fused-mg" else "0")
    return {"fused-mg": 3, "fused": 2, "separate": 1}[request.param]


@pytest.mark.parametrize("value_mode", [0, 1])
@pytest.mark.parametrize("B", [1, 7, 100, 999, 1000, 1001, 2500, -1])
def test_pm_batch_sizes_and_wraps(pm_on, B, value_mode):
    # unit (value_mode 0: no value arrays) and fp32 values; batches that
    # divide N, wrap at the epoch end, or wrap twice (B > N)
    D = 30000
    ds = dlr.Dataset.generate(1000, D, 20, value_mode=value_mode, seed=3, stream=1)
    # the margin in the gradient's launch (3) needs the LDS-phase gradient
    # (row-round batches, small B, keep pass 2 a launch of its own: 2) and
    # every 64-row block summed by a wave of the launch: blocks <= slices x
    # the waves that fill the residuals (B = 2,500 > N: 40 blocks, 8 slices
    # x 1 -> 2)
    Beff = 1000 if B < 0 else B
    fill = 1 if Beff <= 4096 else 2 if Beff <= 8192 else 4 if Beff <= 16384 else 8
    # (a row-round batch keeps pass 2 a launch of its own below 2 rounds)
    rounds = _rounds_of(ds, D, B)
    fits = (Beff + 63) // 64 <= (D + 4095) // 4096 * (5 if rounds else fill) and rounds != 1
    assert _mode_of(ds, D, B) == (2 if pm_on == 3 and not fits else pm_on)
    eng = run_engine([ds], D, 3, B, 0.1)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 3, B, 0.1)
    compare_runs(eng, orc)


def test_pm_ragged_empty_and_long_rows(pm_on):
    # rows of 0..99 entries (the slot lists of a block: up to 13 groups of 8)
    D = 300_000
    ds = _ragged(7, D, 3000)
    test = _ragged(8, D, 500)
    eng = run_engine([ds], D, 3, 257, 0.3, test=test, test_interval=1)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 3, 257, 0.3, test=oracle_shard(test, D), test_interval=1)
    compare_runs(eng, orc)


def test_pm_rows_too_long_fall_back(monkeypatch):
    # a row over 128 entries does not fit the slot lists: DLR_PM=1 is an
    # error, the default quietly keeps the gather margin
    D = 5000
    ds = dlr.Dataset.generate(300, D, 200, value_mode=1, seed=5, stream=1)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    with pytest.raises(dlr.DLRError, match="product margin"):
        _mode_of(ds, D, 64)
    monkeypatch.delenv("DLR_PM")
    assert _mode_of(ds, D, 64) == 0


def test_pm_guess_misses_and_weight_changes(monkeypatch):
    # The fused gradient forms the products of batch b+1: steps out of order,
    # repeated batches, set_weights and predict between steps must all give
    # the gather margin's bits (DLR_PM=0, same sequence).
    D = 300_000
    ds = dlr.Dataset.generate(2000, D, 24, value_mode=1, seed=11, stream=1)
    test = dlr.Dataset.generate(300, D, 24, value_mode=1, seed=11, stream=2)
    rng = np.random.default_rng(3)
    nb = 4
    order = [0, 1, 2, 3, 0, 2, 2, 1, 3, 0, 0, 1, 2, 3]
    perturb = {5: rng.standard_normal(D).astype(np.float32) * np.float32(0.01), 9: None}

    def run(pm):
        monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
        monkeypatch.setenv("DLR_PM", pm)
        eng = dlr.Engine(D)
        try:
            eng.set_weights(dlr.init_weight(D))
            assert eng.load_train(ds, 500) == nb
            eng.load_test(test)
            assert eng.train_product_margin() == (2 if pm == "1" else 0)  # one row round: pass 2 separate
            out = []
            for k, b in enumerate(order):
                if k in perturb:
                    w = eng.get_weights()
                    if perturb[k] is not None:
                        eng.set_weights(w + perturb[k])
                    else:
                        out.append(eng.predict())
                eng.train_step(b, 0.2, 1.0)
                out.append(eng.get_weights())
            return out
        finally:
            eng.close()

    got, ref = run("1"), run("0")
    for a, b in zip(got, ref):
        if isinstance(a, tuple):
            assert a == b
        else:
            assert_same_weights(a, b)


@pytest.mark.parametrize("mode", [dlr.MODE_SYNC_MEAN, dlr.MODE_SYNC_LAST, dlr.MODE_ASYNC])
@pytest.mark.parametrize("W", [2, 3])
def test_pm_world_gt_1(pm_on, W, mode):
    # world > 1 (loopback group): the gradient is not fused with the update,
    # so pass 1 runs on its own every step (mode 1 whatever DLR_PM_FUSED)
    D = 200_000
    shards = [dlr.Dataset.generate(1200, D, 18, value_mode=1, seed=13, stream=r + 1) for r in range(W)]
    eng = run_group(shards, D, 2, 300, 0.2, mode=mode)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 300, 0.2, mode=mode)
    assert_same_weights(eng.w, orc.w)


@pytest.mark.parametrize("W", [2, 5])
def test_pm_exchange_overlap_on_off(monkeypatch, W):
    # the all-gather in pieces with the next batch's pass 1 formed slice
    # group by slice group as the weights land (default), against the plain
    # all-gather: the same bits, the oracle's; D = 300,000 gives key ranges
    # that cut 4,096-column slices (a slice completes only when every range
    # it overlaps has delivered its piece)
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    D = 300_000
    shards = [dlr.Dataset.generate(1500, D, 20, value_mode=1, seed=19, stream=r + 1) for r in range(W)]
    seen = []

    def setup(on):
        def f(eng):
            eng.set_exchange_overlap(on)
            seen.append((eng.train_product_margin(), eng.exchange_overlap()))
        return f

    got = {on: run_group(shards, D, 2, 250, 0.2, setup=setup(on), preload=lambda eng, r: eng.set_exchange_pieces(4))
           for on in (True, False)}
    assert (1, True) in seen and (1, False) in seen
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 250, 0.2)
    assert_same_weights(got[True].w, orc.w, "overlapped exchange")
    assert_same_weights(got[False].w, orc.w, "plain all-gather")


@pytest.mark.parametrize("loop", ["async", "sync"])
@pytest.mark.parametrize("pieces", [1, 3, 16])
def test_pm_exchange_pieces(monkeypatch, pieces, loop):
    # the piece count of the overlapped all-gather (dlr_set_exchange_pieces,
    # a load-time setting), under the stream-ordered loopback collectives
    # (default: copies wait on the peers' events, as RCCL's) and the
    # synchronous ones: the oracle's bits whatever the pieces
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    monkeypatch.setenv("DLR_LOOPBACK_SYNC", "1" if loop == "sync" else "0")
    D, W = 300_000, 3
    shards = [dlr.Dataset.generate(1500, D, 20, value_mode=1, seed=29, stream=r + 1) for r in range(W)]
    seen = []

    def pre(eng, r):
        eng.set_exchange_pieces(pieces)

    def setup(eng):
        seen.append(eng.exchange_pieces())

    got = run_group(shards, D, 2, 250, 0.2, setup=setup, preload=pre)
    assert seen == [pieces] * W
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 250, 0.2)
    assert_same_weights(got.w, orc.w, f"{pieces} pieces, {loop} loopback")


@pytest.mark.parametrize("loop", ["async", "sync"])
def test_pm_exchange_form_agreed_over_ranks(monkeypatch, loop):
    # one rank asks for the plain all-gather before loading, the others for
    # the pieced one (4 pieces): the ranks agree at load on the plain
    # form (the two forms are different collective sequences),
    # every rank reports it, and the weights are the oracle's
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    monkeypatch.setenv("DLR_LOOPBACK_SYNC", "1" if loop == "sync" else "0")
    D, W = 300_000, 3
    shards = [dlr.Dataset.generate(1500, D, 20, value_mode=1, seed=47, stream=r + 1) for r in range(W)]
    seen = []

    def pre(eng, r):
        eng.set_exchange_pieces(4)
        if r == 1:
            eng.set_exchange_overlap(False)

    got = run_group(shards, D, 2, 250, 0.2, preload=pre,
                    setup=lambda eng: seen.append((eng.train_product_margin(), eng.exchange_overlap())))
    assert len(seen) == W and all(pm == 1 and not ov for pm, ov in seen), seen
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 250, 0.2)
    assert_same_weights(got.w, orc.w, "agreed plain all-gather")


def test_pm_exchange_pieces_must_agree(monkeypatch):
    # ranks asking for different piece counts: every rank's load fails
    # (the pieces are collectives), none hangs
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    D, W = 50_000, 2
    shards = [dlr.Dataset.generate(400, D, 10, value_mode=1, seed=31, stream=r + 1) for r in range(W)]
    with pytest.raises(dlr.DLRError, match="piece counts"):
        run_group(shards, D, 1, 100, 0.2, preload=lambda eng, r: eng.set_exchange_pieces(2 + r))
    eng = dlr.Engine(D)
    try:
        for bad in (-1, 17):
            with pytest.raises(dlr.DLRError):
                eng.set_exchange_pieces(bad)
        eng.set_exchange_pieces(0)  # auto (the default)
    finally:
        eng.close()


@pytest.mark.parametrize("W", [2, 8])
def test_pm_exchange_auto_pieces_is_one_gather(monkeypatch, W):
    # the default piece count is one per 4 MiB of a rank's key range: a
    # C2-sized D (<= 4 MB of weights) gets ONE piece, i.e. no overlap -- the
    # plain in-place all-gather, not W - 1 sends and receives per piece --
    # bitwise the oracle
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    D = 300_000
    shards = [dlr.Dataset.generate(900, D, 12, value_mode=1, seed=41, stream=r + 1) for r in range(W)]
    seen = []
    got = run_group(shards, D, 2, 200, 0.2, setup=lambda eng: seen.append((eng.exchange_overlap(), eng.exchange_pieces())))
    assert seen == [(0, 0)] * W
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 200, 0.2)
    compare_runs(got, orc)


def test_pm_overlap_through_rccl_one_rank(monkeypatch):
    # the RCCL transport's pieced all-gather (grouped send/recv; no peers at
    # one rank) with every slice in this rank's own range: the same bits
    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    D = 300_000
    ds = dlr.Dataset.generate(1500, D, 20, value_mode=1, seed=23, stream=1)
    eng = run_engine([ds], D, 2, 250, 0.2)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 2, 250, 0.2)
    compare_runs(eng, orc)


def test_rccl_abort_from_another_thread(monkeypatch):
    # dlr_comm_abort on an RCCL communicator from a thread that does not
    # drive it (bin/distlr's in-process topology aborts every rank's
    # communicator from the failing rank's thread): it only flags the
    # communicator; the driving thread's next stream wait or collective
    # aborts it (ncclCommAbort) and fails with the reason, and the context
    # still closes
    import threading

    monkeypatch.setenv("DLR_FORCE_COLLECTIVES", "1")
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    D = 300_000
    ds = dlr.Dataset.generate(1500, D, 20, value_mode=1, seed=43, stream=1)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        nb = eng.load_train(ds, 250)
        eng.train_step(0, 0.2, 1.0)
        eng.sync()
        th = threading.Thread(target=eng.comm_abort, args=("rank 0 lost its shard",))
        th.start()
        th.join()
        with pytest.raises(dlr.DLRError, match="lost its shard"):
            for b in range(1, nb):
                eng.train_step(b, 0.2, 1.0)
            eng.sync()
    finally:
        eng.close()


def test_pm_parameter_server_topology(pm_on):
    # W workers through dlr_worker_gradient / dlr_server_apply
    D = 200_000
    shards = [dlr.Dataset.generate(1200, D, 18, value_mode=1, seed=17, stream=r + 1) for r in range(2)]
    eng = run_engine(shards, D, 2, 300, 0.2)
    orc = oracle.run_worker([oracle_shard(s, D) for s in shards], D, 2, 300, 0.2)
    compare_runs(eng, orc)


def test_pm_default_on_c2_shape():
    # The headline shape turns the product margin on by default (245 column
    # slices); two epochs + a step vs the gather margin and the oracle.
    D = 1_000_000
    ds = dlr.Dataset.generate(200_000, D, 50, value_mode=1, seed=12, stream=1)
    rp, col, val, lab = ds.csr()
    w0 = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w0)
        nb = eng.load_train(ds, 65536)
        assert eng.train_layout() == dlr.LAYOUT_LDS and eng.train_product_margin() == 3
        w = w0.copy()
        for b in range(2 * nb + 1):
            bb = b % nb
            eng.train_step(bb, 0.2, 1.0)
            g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(len(lab), 65536, bb), w)
            oracle.server_update(w, [g], 0.2)
        assert_same_weights(eng.get_weights(), w)
    finally:
        eng.close()


@pytest.mark.parametrize("rt", ["1", "0"])
@pytest.mark.parametrize("B", [8192, 20000, 40000, 65536])
def test_pm_row_round_gradient(monkeypatch, rt, B):
    # the row-round gradient (k_grad_rt: 1 to 8 rounds of 8,192 rows; the
    # pass-1 list issued by rounds 4+ or after the last of <= 3 rounds; the
    # margin's pass 2 in the same launch from 2 rounds, k_grad_rt MG) against k_grad_lds
    # and the oracle's sparse step: bitwise either way, fused pass 1,
    # wrapping batches
    monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
    monkeypatch.setenv("DLR_PM", "1")
    monkeypatch.setenv("DLR_GRAD_RT", rt)
    D = 1 << 20
    ds = dlr.Dataset.generate(70_000, D, 20, value_mode=1, seed=11, stream=1)
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    eng = dlr.Engine(D)
    try:
        eng.set_weights(w)
        nb = eng.load_train(ds, B)
        # (pass 2 in the gradient's launch; one row round keeps it separate)
        assert eng.train_product_margin() == (2 if rt == "1" and B <= 8192 else 3)
        assert eng.train_row_rounds() == ((B + 8191) // 8192 if rt == "1" else 0)
        for b in range(nb + 1):  # an epoch (the last batch wraps) + the next epoch's first
            eng.train_step(b % nb, 0.2, 1.0)
            g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(len(lab), B, b % nb), w)
            oracle.server_update(w, [g], 0.2)
        assert_same_weights(eng.get_weights(), w)
    finally:
        eng.close()


@pytest.mark.parametrize("B", [20000, 65536])
def test_pm_margin_in_gradient_launch(monkeypatch, B):
    # Pass 2 inside the fused gradient's launch (dlr_train_product_margin 3,
    # k_grad_lds MG): ragged rows of 0..64 entries (empty rows, whole empty
    # 64-row blocks), a wrapping last batch, steps out of order and repeated,
    # set_weights between steps (the products are re-formed: a guess missed)
    # -- bitwise the separate pass 2 (DLR_PM_MG=0) and the oracle.
    D = 1 << 20
    rng = np.random.default_rng(21)
    n = 150_000
    lens = rng.integers(0, 65, size=n)
    lens[rng.choice(n, 5000, replace=False)] = 0
    lens[64 * 100:64 * 102] = 0  # two empty blocks
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(D, k, replace=False)) for k in lens]).astype(np.int32)
    val = rng.integers(1, 10001, size=len(col)).astype(np.float32) / np.float32(10000)
    lab = rng.integers(0, 2, size=n).astype(np.int32)
    ds = dlr.Dataset.from_csr(rp, col, val, lab, D)
    w0 = dlr.init_weight(D)
    order = [0, 1, 2, 2, 0, 1, 1, 2, 0]
    bump = {4: rng.standard_normal(D).astype(np.float32) * np.float32(0.01)}

    def run(mg):
        monkeypatch.setenv("DLR_GRAD_KERNEL", "lds")
        monkeypatch.setenv("DLR_PM", "1")
        monkeypatch.setenv("DLR_PM_MG", mg)
        eng = dlr.Engine(D)
        try:
            eng.set_weights(w0)
            nb = eng.load_train(ds, B)
            assert eng.train_product_margin() == (3 if mg == "1" else 2)
            assert eng.train_row_rounds() == 0
            out = []
            for k, b in enumerate(order):
                if k in bump:
                    eng.set_weights(eng.get_weights() + bump[k])
                eng.train_step(b % nb, 0.2, 1.0)
                out.append(eng.get_weights())
            return out, nb
        finally:
            eng.close()

    (got, nb), (ref, _) = run("1"), run("0")
    for a, b in zip(got, ref):
        assert_same_weights(a, b)
    w = w0.copy()
    for k, b in enumerate(order):
        if k in bump:
            w = w + bump[k]
        g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b % nb), w)
        oracle.server_update(w, [g], 0.2)
    assert_same_weights(got[-1], w)


@pytest.mark.parametrize("band_rows", ["262144", "524288"])
def test_pm_windows_full_shard_batch(monkeypatch, band_rows):
    # B = -1 over > 2^20 rows (band mode): the margin as
    # the product margin over 65,536-row windows -- pass 1 and pass 2 per
    # window, the weights fixed inside the step (dlr_train_product_margin 1)
    # -- two steps, bitwise the gather margin (DLR_PM=0) and the oracle
    monkeypatch.setenv("DLR_BAND_ROWS", band_rows)
    D = 1 << 20
    n = 1_100_000
    ds = dlr.Dataset.generate(n, D, 50, value_mode=1, seed=8, stream=3)

    def run(pm):
        monkeypatch.setenv("DLR_PM", pm)
        eng = dlr.Engine(D)
        try:
            eng.set_weights(dlr.init_weight(D))
            assert eng.load_train(ds, -1) == 1
            assert eng.train_band_rows() == int(band_rows)
            kind = eng.train_product_margin()
            for _ in range(2):
                eng.train_step(0, 0.2, 1.0)
            return eng.get_weights(), kind
        finally:
            eng.close()

    got, kind = run("1")
    assert kind == 1
    ref, kind0 = run("0")
    assert kind0 == 0
    assert_same_weights(got, ref, "windowed product margin vs gathers")
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    for _ in range(2):
        g = oracle.grad_csr((rp, col, val), lab, np.arange(n), w)
        oracle.server_update(w, [g], 0.2)
    assert_same_weights(got, w, "windowed product margin vs oracle")


def test_pm_windows_wrapping_batches(monkeypatch):
    # Band mode with batches that are not the whole shard: B = 600,000 over
    # 1.1M rows in 2^18-row bands -- per batch 2 full bands (4 windows each,
    # one pass-1 and one pass-2 launch a band) and a 75,712-row band (2
    # windows, the last partial); batch 1 wraps to row 0 (data_iter.h:49-52).
    # Three steps (batches 0, 1, 0), bitwise the gather margin and the oracle.
    monkeypatch.setenv("DLR_BAND_ROWS", "262144")
    D, n, B = 1 << 20, 1_100_000, 600_000
    ds = dlr.Dataset.generate(n, D, 50, value_mode=1, seed=9, stream=5)
    seq = [0, 1, 0]

    def run(pm):
        monkeypatch.setenv("DLR_PM", pm)
        eng = dlr.Engine(D)
        try:
            eng.set_weights(dlr.init_weight(D))
            assert eng.load_train(ds, B) == 2
            assert eng.train_band_rows() == 262144
            kind = eng.train_product_margin()
            for b in seq:
                eng.train_step(b, 0.2, 1.0)
            return eng.get_weights(), kind
        finally:
            eng.close()

    got, kind = run("1")
    assert kind == 1
    ref, _ = run("0")
    assert_same_weights(got, ref, "windowed product margin vs gathers (wrapping batches)")
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    for b in seq:
        g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(n, B, b), w)
        oracle.server_update(w, [g], 0.2)
    assert_same_weights(got, w, "windowed product margin vs oracle (wrapping batches)")


def _strided_of(ds, D, B):
    eng = dlr.Engine(D)
    try:
        eng.set_weights(dlr.init_weight(D))
        eng.load_train(ds, B)
        return eng.train_product_margin(), eng.train_pm_strided()
    finally:
        eng.close()


@pytest.mark.parametrize("shape", ["uniform", "ragged"])
def test_pm_region_strides(pm_on, shape):
    # The product margin's regions and slot lists at fixed strides (uniform
    # rows: pass 2 loads no offsets first) and packed (ragged rows: the
    # largest region is far above the mean), every pass-2 form (pm_on):
    # both bitwise the oracle.
    D = 300_000
    if shape == "uniform":
        ds = dlr.Dataset.generate(3000, D, 50, value_mode=1, seed=11, stream=2)
    else:
        ds = _ragged(9, D, 3000, max_len=90)  # (a block's region stays within kPmCap)
    B = 1024
    mode, strided = _strided_of(ds, D, B)
    assert mode > 0
    # (ragged: 0, or 2 if some batch's blocks happen to be even)
    assert strided == 1 if shape == "uniform" else strided in (0, 2), strided
    eng = run_engine([ds], D, 3, B, 0.2)
    orc = oracle.run_worker([oracle_shard(ds, D)], D, 3, B, 0.2)
    compare_runs(eng, orc)
