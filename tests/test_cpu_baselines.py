"""The CPU baselines bench.py reports (oracle/cpu_baselines.py), checked on
CPU: the reference-structure run (local.sh topology, O(B*D^2) loop, per-
epoch re-parse) must produce the oracle's frozen trajectories bitwise --
it does the reference's work AND gets the reference's bits -- and the
OpenMP "build CPU path, not reference" must train the same model within a
tolerance (its sums are reordered across threads)."""
from __future__ import annotations

import os

import numpy as np
import pytest

import cpu_baselines as cb
import distlr_amd as dlr
import oracle
from conftest import GOLDEN, read_golden_json


@pytest.mark.parametrize("name", list(read_golden_json("trajectories.json")))
def test_reference_structure_run_matches_golden(name):
    meta = read_golden_json("trajectories.json")[name]
    root = os.path.join(GOLDEN, meta["dataset"])
    w, steps, sec, correct, rows = cb.reference_local_run(root, meta["workers"], meta["D"], meta["num_iteration"],
                                                          meta["batch_size"], meta["test_interval"],
                                                          meta["learning_rate"], meta["mode"])
    assert w.astype("<f4").tobytes().hex() == meta["w"]
    assert (correct, rows) == tuple(meta["tests"][-1][1:3])
    n = sum(len(open(os.path.join(root, "train", f"part-00{r + 1}")).read().splitlines())
            for r in range(meta["workers"]))
    per_epoch = sum(oracle.num_batches(len(open(os.path.join(root, "train", f"part-00{r + 1}")).read().splitlines()),
                                       meta["batch_size"]) * (meta["batch_size"] if meta["batch_size"] > 0 else
                                                               len(open(os.path.join(root, "train",
                                                                                     f"part-00{r + 1}")).read()
                                                                   .splitlines()))
                    for r in range(meta["workers"]))
    assert n > 0 and steps == per_epoch * meta["num_iteration"] and sec > 0


def test_reference_inner_cost_scales_with_D():
    small = cb.reference_inner_cost(1000, 4, 20000)
    big = cb.reference_inner_cost(100_000, 4, 200)
    assert 0 < small < big


def _csr(ds):
    rp, col, val, lab = ds.csr()
    return rp, col, val, lab


@pytest.mark.parametrize("unit", [False, True])
@pytest.mark.parametrize("B", [64, 1000, -1])
def test_omp_csr_close_to_oracle(unit, B):
    D = 2000
    ds = dlr.Dataset.generate(3000, D, 20, value_mode=0 if unit else 1, seed=4, stream=1)
    rp, col, val, lab = _csr(ds)
    w = dlr.init_weight(D)
    wo = w.copy()
    nb = oracle.num_batches(len(lab), B)
    steps = 2 * nb
    cb.omp_train_csr(rp, col, None if unit else val, lab, D, B, w, 0.2, 1.0, 0, steps)
    for s in range(steps):
        g = oracle.grad_csr((rp, col, val), lab, oracle.batch_rows(len(lab), B, s % nb), wo)
        oracle.server_update(wo, [g], 0.2)
    assert np.allclose(w, wo, rtol=1e-4, atol=1e-6)


def test_omp_dense_close_to_oracle():
    D, B = 256, 500
    dd = dlr.DenseDataset.generate(1200, D, seed=5, stream=1)
    X, y = dd.arrays()
    w = dlr.init_weight(D)
    wo = w.copy()
    nb = oracle.num_batches(len(y), B)
    cb.omp_train_dense(X, y, B, w, 0.05, 1.0, 0, 2 * nb)
    for s in range(2 * nb):
        g = oracle.grad_dense(X, y, oracle.batch_rows(len(y), B, s % nb), wo)
        oracle.server_update(wo, [g], 0.05)
    assert np.allclose(w, wo, rtol=1e-4, atol=1e-6)
    assert cb.omp_threads() >= 1
