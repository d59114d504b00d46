"""The committed PMC traffic figures (profiles/traffic*.json, which bench.py
reports as roofline.traffic) must be reproducible from the committed raw
rocprofv3 counter CSVs (profiles/r02_pmc_<config>/) with tools/pmc_traffic.py
-- no figure in the bench line without its raw data."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    # round 5: the margin in the gradient's launch (one launch per step),
    # the round-5 issue order
    ("traffic.json", "r06_pmc_c2", "D1000000_nnz50_B65536", "lds", 0),
    # round 5: C3 in the reference order (hot-column product stream); 14
    # step-equivalents (bench --steps 6 --warmup 2 --no-stage-pass: 2 + 6 +
    # 6 steps)
    ("traffic_c3.json", "r06_pmc_c3", "D16777216_nnz39_B-1", "classic", 14),
    # round 3: C3 in the FAST order (c3f); the band-pipelined margin is
    # dispatched per band; 20 step-equivalents (bench --steps 6 --warmup 2:
    # 2 + 6 timed + 6 + 6 stage and breakdown steps)
    ("traffic_c3f.json", "r03_pmc_c3", "D16777216_nnz39_B-1", "classic", 20),
    # round 4: C4 in the reference order (K6r, one launch per step)
    ("traffic_c4.json", "r04_pmc_c4", "D4096_nnz4096_B65536", "dense", 0),
    ("traffic_c5.json", "r02_pmc_c5", "D268435456_nnz10_B1024", "touched", 0),
]


@pytest.mark.parametrize("name,raw,key,layout,steps", CASES)
def test_traffic_reproducible_from_raw_counters(name, raw, key, layout, steps):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"),
                          os.path.join(ROOT, "profiles", raw), "--workload-key", key, "--layout", layout,
                          "--steps", str(steps)],
                         check=True, capture_output=True, text=True).stdout
    got = json.loads(out)
    with open(os.path.join(ROOT, "profiles", name)) as f:
        want = json.load(f)
    assert got["workload_key"] == want["workload_key"] == key
    assert got["hbm_bytes_per_step"] == want["hbm_bytes_per_step"]
    assert got["hbm_bytes_per_step"] > 0
    # the read correction is the measured gfx950 factor (~2: FETCH_SIZE counts
    # half of a wide streaming read), not an assumed constant
    assert 1.8 < got["calibration"]["read_factor"] < 2.2
