"""End to end through the C++ drop-in: bin/distlr (the main.cc replacement)
with local.sh's environment, against the oracle's frozen trajectories:
accuracy lines and every worker's model file (lr.cc:73-82 text of the last
pulled weights)."""
from __future__ import annotations

import os
import shutil
import subprocess

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, ROOT, read_golden_json

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "dist-lr_amd", "bin", "distlr")


def run_distlr(tmp_path, dataset, meta, workers, extra_env=None):
    data = tmp_path / "data"
    shutil.copytree(os.path.join(GOLDEN, dataset), data)
    env = dict(os.environ)
    env.update({
        "DATA_DIR": str(data), "NUM_FEATURE_DIM": str(meta["D"]), "NUM_ITERATION": str(meta["num_iteration"]),
        "BATCH_SIZE": str(meta["batch_size"]), "TEST_INTERVAL": str(meta["test_interval"]), "SYNC_MODE": "1",
        "LEARNING_RATE": repr(meta["learning_rate"]), "DMLC_NUM_WORKER": str(workers), "RANDOM_SEED": "10",
    })
    if extra_env:
        env.update(extra_env)
    r = subprocess.run([BIN], env=env, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    out = r.stdout.decode()
    lines = [l[l.index("Iteration "):] for l in out.splitlines() if " Iteration " in l]
    models = [(data / "models" / f"part-00{r + 1}").read_text() for r in range(workers)]
    return out, lines, models


@pytest.mark.parametrize("name,workers,topo", [("c1_W1_Bfull_mean", 1, None), ("c1_W1_B7_mean", 1, None),
                                               ("c1_W2_Bfull_mean", 2, "group"), ("real_W2_B50_mean", 2, "group"),
                                               ("c1_W2_Bfull_mean", 2, "ps"), ("real_W2_B50_mean", 2, "ps")])
def test_distlr_matches_oracle(tmp_path, name, workers, topo):
    # W = 2 on one GPU: the loopback group (default there) and the
    # parameter-server topology
    meta = read_golden_json("trajectories.json")[name]
    out, lines, models = run_distlr(tmp_path, meta["dataset"], meta, workers,
                                    {"DISTLR_TOPOLOGY": topo} if topo else None)
    assert "Server mode: sync" in out
    lr_env = repr(meta["learning_rate"])
    if np.float32(oracle.to_float(lr_env)) == np.float32(meta["learning_rate"]):
        expect_lines, pulled = meta["accuracy_lines"], [
            np.frombuffer(bytes.fromhex(h), dtype="<f4") for h in meta["pulled"]]
    else:
        # main.cc:27 parses LEARNING_RATE with ToFloat, which is not strtof:
        # ToFloat("0.05") is 0x3D4CCCCC, not 0.05f.  Recompute the oracle run
        # with the rate the reference itself would use.
        base = os.path.join(GOLDEN, meta["dataset"])
        shards = [oracle.load_dense(os.path.join(base, "train", f"part-00{p + 1}"), meta["D"])
                  for p in range(workers)]
        test = oracle.load_dense(os.path.join(base, "test", "part-001"), meta["D"])
        res = oracle.run_worker(shards, meta["D"], meta["num_iteration"], meta["batch_size"],
                                oracle.to_float(lr_env), test=test, test_interval=meta["test_interval"],
                                mode=meta["mode"])
        expect_lines, pulled = res.accuracy_lines(), res.pulled
    assert lines == expect_lines
    for r in range(workers):
        assert models[r] == dlr.format_model(pulled[r]), f"model part-00{r + 1}"


def test_distlr_sync_merge_last(tmp_path):
    meta = read_golden_json("trajectories.json")["c1_W2_Bfull_last"]
    _, lines, models = run_distlr(tmp_path, meta["dataset"], meta, 2, {"DISTLR_SYNC_MERGE": "last"})
    assert lines == meta["accuracy_lines"]
    assert models[0] == meta["model_rank0"]


def test_distlr_forced_rccl_single_worker(tmp_path):
    meta = read_golden_json("trajectories.json")["c1_W1_Bfull_mean"]
    _, lines, models = run_distlr(tmp_path, meta["dataset"], meta, 1, {"DLR_FORCE_COLLECTIVES": "1"})
    assert lines == meta["accuracy_lines"] and models[0] == meta["model_rank0"]


def test_distlr_missing_env_is_reported(tmp_path):
    r = subprocess.run([BIN], env={"PATH": os.environ.get("PATH", "")}, capture_output=True, timeout=60)
    assert r.returncode == 2 and b"DATA_DIR" in r.stderr


LOCAL_SH_PATTERN = """#!/bin/bash
# local.sh's launch pattern (examples/local.sh:11-51): env, then one
# scheduler, $1 servers and $2 workers of the same binary in the background
export DATA_DIR="$3" NUM_FEATURE_DIM=123 LEARNING_RATE=0.2 TEST_INTERVAL=10 SYNC_MODE=1
export NUM_ITERATION=100 BATCH_SIZE=-1 RANDOM_SEED=10
export DMLC_NUM_SERVER=$1 DMLC_NUM_WORKER=$2 DMLC_PS_ROOT_URI=127.0.0.1 DMLC_PS_ROOT_PORT=8001
bin="$4"
export DMLC_ROLE=scheduler; $bin &
export DMLC_ROLE=server; for ((i=0; i<DMLC_NUM_SERVER; ++i)); do $bin & done
export DMLC_ROLE=worker; for ((i=0; i<DMLC_NUM_WORKER; ++i)); do $bin & done
wait
"""


def test_local_sh_roles(tmp_path):
    # local.sh 1 2 bin/distlr: exactly one training run (in the scheduler
    # process), one set of accuracy lines, one server mode line, and the
    # model files of the 2-worker mean run
    data = tmp_path / "data"
    shutil.copytree(os.path.join(GOLDEN, "c1_tiny"), data)
    # local.sh's own settings (100 epochs, B = -1, test every 10, lr 0.2)
    D = 123
    shards = [oracle.load_dense(str(data / "train" / f"part-00{p + 1}"), D) for p in range(2)]
    test = oracle.load_dense(str(data / "test" / "part-001"), D)
    orc = oracle.run_worker(shards, D, 100, -1, oracle.to_float("0.2"), test=test, test_interval=10)
    script = tmp_path / "local_pattern.sh"
    script.write_text(LOCAL_SH_PATTERN)
    r = subprocess.run(["bash", str(script), "1", "2", str(data), BIN], capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    out = r.stdout.decode()
    lines = [l[l.index("Iteration "):] for l in out.splitlines() if " Iteration " in l]
    assert lines == orc.accuracy_lines() and len(lines) == 10
    assert out.count("Server mode: sync") == 1
    assert out.count("Worker[0]: start working...") == 1 and out.count("Worker[1]: start working...") == 1
    for rk in range(2):
        assert (data / "models" / f"part-00{rk + 1}").read_text() == dlr.format_model(orc.pulled[rk])


def test_unknown_role_is_reported(tmp_path):
    env = {"PATH": os.environ.get("PATH", ""), "DATA_DIR": str(tmp_path), "NUM_FEATURE_DIM": "10",
           "NUM_ITERATION": "1", "BATCH_SIZE": "-1", "TEST_INTERVAL": "1", "SYNC_MODE": "1", "LEARNING_RATE": "0.1",
           "DMLC_ROLE": "bogus"}
    r = subprocess.run([BIN], env=env, capture_output=True, timeout=60)
    assert r.returncode == 2 and b"DMLC_ROLE" in r.stderr


@pytest.mark.parametrize("B,k", [(7, 3), (64, 100), (-1, 5), (3000, 1)])
def test_train_on_partially_consumed_dataiter(B, k):
    # lr.cc:29-30 trains what is left of the round: after NextBatch(k) the
    # batches start at row k and wrap to row 0 (data_iter.h:49-52), and
    # Train stops after the batch that ends the round.  Against the oracle's
    # sequential sums for exactly those rows; the iterator ends where
    # NextBatch would leave it; GetWeight is the last PULLED weights (the
    # ones before the last batch's update, lr.cc:32).
    tool = os.path.join(ROOT, "dist-lr_amd", "bin", "distlr_tool")
    path = os.path.join(GOLDEN, "c1_tiny", "train", "part-001")
    D, lr = 123, 0.2
    r = subprocess.run([tool, "partial", path, str(D), str(B), str(k), repr(lr)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    out = r.stdout.decode().split()
    n_rows = dlr.Dataset.load_libsvm(path, D).n_rows
    assert out[0:3] == ["before", str(k % n_rows), "1" if k < n_rows else "0"]
    got = np.array([int(x, 16) for x in out[6:]], dtype=np.uint32).view(np.float32)
    bs = n_rows if B < 0 else B
    nb = -(-(n_rows - k) // bs)
    assert out[3:6] == ["after", str((k + nb * bs) % n_rows), "0"]
    ds = dlr.Dataset.load_libsvm(path, D)
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    pulled = w.copy()
    for m in range(nb):
        rows = (k + m * bs + np.arange(bs)) % n_rows
        pulled = w.copy()
        oracle.server_update(w, [oracle.grad_csr((rp, col, val), lab, rows, w)], lr)
    assert np.array_equal(got.view(np.uint32), pulled.view(np.uint32))
