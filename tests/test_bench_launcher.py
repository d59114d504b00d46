"""bench.py's own launcher (no torch.distributed.run): the parent starts one
process per rank with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and never
touches a GPU; the ranks rendezvous over gloo (CPU check, no GPU work)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True,
                          timeout=300, env=env)


def test_launcher_spawns_ranks():
    r = _run("--gpus", "3", "--launcher-check")
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    out = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert out["world"] == 3
    assert [x["rank"] for x in out["launcher_check"]] == [0, 1, 2]
    assert [x["local_rank"] for x in out["launcher_check"]] == [0, 1, 2]
    assert len({x["pid"] for x in out["launcher_check"]}) == 3


def test_launcher_at_one_gpu():
    r = _run("--gpus", "1", "--spawn", "--launcher-check")
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    out = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert out["world"] == 1 and out["launcher_check"][0]["rank"] == 0
