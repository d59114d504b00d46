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
    lines = [l.split(" ", 1)[1] for l in out.splitlines() if " Iteration " in l]
    models = [(data / "models" / f"part-00{r + 1}").read_text() for r in range(workers)]
    return out, lines, models


@pytest.mark.parametrize("name,workers", [("c1_W1_Bfull_mean", 1), ("c1_W1_B7_mean", 1),
                                          ("c1_W2_Bfull_mean", 2), ("real_W2_B50_mean", 2)])
def test_distlr_matches_oracle(tmp_path, name, workers):
    meta = read_golden_json("trajectories.json")[name]
    out, lines, models = run_distlr(tmp_path, meta["dataset"], meta, workers)
    assert "Server mode: sync" in out
    assert lines == meta["accuracy_lines"]
    for r in range(workers):
        pulled = np.frombuffer(bytes.fromhex(meta["pulled"][r]), dtype="<f4")
        assert models[r] == dlr.format_model(pulled), f"model part-00{r + 1}"


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
