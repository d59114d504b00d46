#!/usr/bin/env python3
"""make_golden.py -- regenerates the golden fixtures under tests/golden/.

Runs ONLY in the build container (it needs /root/reference for the
reference-built driver oracle/_ref/ref_driver; `make -C oracle` builds it).
The fixtures it writes are data (inputs + expected outputs) and travel with
the repo; nothing here is needed at test time.

Sources of truth
  kat.tsv, *.parse.sha256, *.batches.*  <- oracle/_ref/ref_driver, i.e. the
      reference's own util.cc + data_iter.h + sample.h compiled as they lie.
  rand_kat.json                         <- glibc srand/rand (the reference's
      dependency, lr.cc:92-98) called through ctypes.
  trajectories.json                     <- the oracle restatement
      (oracle/lr_oracle.c; LR arithmetic is "parity unpinned" by reference
      execution) -- freezes it against regressions.
Input data files are produced by the product's seeded generator (their
origin does not matter: they are committed and the expected outputs come
from the sources above).
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "dist-lr_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import distlr_amd as dlr  # noqa: E402
import oracle  # noqa: E402

REF = oracle.REF_DRIVER

KAT_STRINGS = [
    "0", "1", "+1", "-1", "2", "10", "123", "-0", "+0", "007", "1.0", "0.5", "0.333333", "0.1234", "1.0000",
    "12.125", "3.14159", "-0.5", "1e-3", "1E5", "1.2.3", "..", ".", "", "a", "abc", "a:b", "a:b:c", "a:b:c:d",
    "1:2:3", "5:1:2:3", "::", ":x", "x:", "99999999999", "2147483648", "-2147483648", "4294967296",
    "0.0001", "0.9999", "0.00000001", "123456789.123456789", "65536.5", " 1", "1 ", "\t2", "1\r",
    "12:0.5", "1:1", "123:1", "0:0", "-5:0.25",
]


def sh(*args) -> str:
    return subprocess.run(list(args), check=True, capture_output=True).stdout.decode("latin-1")


def sha(text: str) -> str:
    return hashlib.sha256(text.encode("latin-1")).hexdigest()


def f32hex(a: np.ndarray) -> str:
    return np.ascontiguousarray(a, dtype="<f4").tobytes().hex()


def write_quirks(path: str) -> None:
    lines = [
        b"+1 3:1 1:0.5 3:2.25",           # duplicate index: last wins; unsorted
        b"",                              # blank: label from previous token "3:2.25"
        b"-1 2:1e-3 4:-0.5",              # ToFloat quirks
        b"   ",                           # whitespace-only: previous token "4:-0.5"
        b"1",                             # label only
        b"",                              # blank after "1": label 1
        b"0 5:1:2:3 6:0 6:7",             # multi-colon Split; explicit zero then dup
        b"+1\t7:12.125\r",                # tab + CRLF
        b"2 8:1.2.3 9:0.0001 10:1.0",     # second '.', tiny value, last column
        b"-1 1:1 2:1 3:1 4:1 5:1 6:1 7:1 8:1 9:1 10:1",
        b"+1 10:5 9:4 8:3 7:2 6:1",       # descending indices
        b"  +1 2:0.1 ",                   # leading/trailing blanks
    ]
    with open(path, "wb") as f:
        f.write(b"\n".join(lines) + b"\n")


def gen_files(base: str, D: int, parts: int, rows: int, test_rows: int, nnz: int, value_mode: int, seed: int):
    os.makedirs(os.path.join(base, "train"), exist_ok=True)
    os.makedirs(os.path.join(base, "test"), exist_ok=True)
    os.makedirs(os.path.join(base, "models"), exist_ok=True)
    files = []
    for p in range(parts):
        ds = dlr.Dataset.generate(rows, D, nnz, value_mode=value_mode, seed=seed, stream=p + 1)
        path = os.path.join(base, "train", f"part-00{p + 1}")
        ds.write_libsvm(path, value_mode)
        files.append(path)
    ds = dlr.Dataset.generate(test_rows, D, nnz, value_mode=value_mode, seed=seed, stream=100)
    path = os.path.join(base, "test", "part-001")
    ds.write_libsvm(path, value_mode)
    files.append(path)
    with open(os.path.join(base, "models", ".keep"), "w"):
        pass
    return files


def main() -> None:
    if not os.path.exists(REF):
        sys.exit(f"{REF} missing: run `make -C oracle` in the build container (needs /root/reference)")
    out = {"generated_by": "tests/golden/make_golden.py", "parse": {}, "batches": {}}

    # 1. ToInt / ToFloat / Split known answers from the reference's util.cc.
    kat_in = os.path.join(HERE, "kat_strings.txt")
    with open(kat_in, "w") as f:
        f.write("\n".join(KAT_STRINGS) + "\n")
    kat = sh(REF, "kat", kat_in)
    with open(os.path.join(HERE, "kat.tsv"), "w") as f:
        f.write(kat)

    # 2. Parse + batching of a hand-written quirks file (full text kept).
    qdir = os.path.join(HERE, "quirks")
    os.makedirs(qdir, exist_ok=True)
    qpath = os.path.join(qdir, "quirks.libsvm")
    write_quirks(qpath)
    with open(os.path.join(qdir, "quirks.parse.txt"), "w") as f:
        f.write(sh(REF, "parse", qpath, "10"))
    for B in (3, 5, -1, 25):
        with open(os.path.join(qdir, f"quirks.batches_B{B}.txt"), "w") as f:
            f.write(sh(REF, "batches", qpath, "10", str(B)))

    # 3. Small gen_data-shaped shards (C1-like) + reference parse digests.
    c1 = os.path.join(HERE, "c1_tiny")
    c1_files = gen_files(c1, 123, 2, 600, 400, 14, 0, seed=10)
    cr = os.path.join(HERE, "c1_real")
    cr_files = gen_files(cr, 64, 2, 300, 200, 9, 1, seed=11)
    for path, D in [(p, 123) for p in c1_files] + [(p, 64) for p in cr_files]:
        rel = os.path.relpath(path, HERE)
        txt = sh(REF, "parse", path, str(D))
        out["parse"][rel] = {"D": D, "n": int(txt.split("\n", 1)[0].split()[1]), "sha256": sha(txt)}
    for B in (7, 100, 600, -1, 1000):
        txt = sh(REF, "batches", c1_files[0], "123", str(B))
        out["batches"][f"c1_tiny/train/part-001@B{B}"] = {"D": 123, "B": B, "sha256": sha(txt),
                                                          "n_batches": txt.count("batch ")}

    # 4. glibc rand known answers (lr.cc:92-98 uses srand/rand).
    libc = ctypes.CDLL("libc.so.6")
    rk = {}
    for seed in (0, 1, 42, 12345):
        libc.srand(seed)
        rk[str(seed)] = [libc.rand() for _ in range(8)]
    with open(os.path.join(HERE, "rand_kat.json"), "w") as f:
        json.dump(rk, f, indent=1)

    # 5. Oracle trajectories (restatement; see module docstring).
    def load(base, D, parts):
        shards = [oracle.load_dense(os.path.join(base, "train", f"part-00{p + 1}"), D) for p in range(parts)]
        test = oracle.load_dense(os.path.join(base, "test", "part-001"), D)
        return shards, test

    c1s, c1t = load(c1, 123, 2)
    crs, crt = load(cr, 64, 2)
    cases = [
        ("c1_W1_Bfull_mean", "c1_tiny", 123, c1s[:1], c1t, 10, -1, 0.2, oracle.MODE_MEAN, 5),
        ("c1_W1_B7_mean", "c1_tiny", 123, c1s[:1], c1t, 2, 7, 0.2, oracle.MODE_MEAN, 1),
        ("c1_W1_B1000_mean", "c1_tiny", 123, c1s[:1], c1t, 2, 1000, 0.2, oracle.MODE_MEAN, 1),
        ("c1_W2_Bfull_mean", "c1_tiny", 123, c1s, c1t, 10, -1, 0.2, oracle.MODE_MEAN, 5),
        ("c1_W2_Bfull_last", "c1_tiny", 123, c1s, c1t, 10, -1, 0.2, oracle.MODE_LAST, 5),
        ("c1_W2_B64_async", "c1_tiny", 123, c1s, c1t, 2, 64, 0.2, oracle.MODE_ASYNC, 1),
        ("real_W2_B50_mean", "c1_real", 64, crs, crt, 3, 50, 0.05, oracle.MODE_MEAN, 1),
        ("real_W1_B33_mean", "c1_real", 64, crs[:1], crt, 3, 33, 0.5, oracle.MODE_MEAN, 3),
    ]
    traj = {}
    for name, dset, D, shards, test, epochs, B, lr, mode, ti in cases:
        res = oracle.run_worker(shards, D, epochs, B, lr, test=test, test_interval=ti, mode=mode, sparse=True)
        dense = oracle.run_worker(shards, D, epochs, B, lr, test=test, test_interval=ti, mode=mode, sparse=False)
        assert np.array_equal(res.w.view(np.uint32), dense.w.view(np.uint32)), f"{name}: sparse != dense"
        traj[name] = {
            "dataset": dset, "D": D, "workers": len(shards), "num_iteration": epochs, "batch_size": B,
            "learning_rate": lr, "mode": mode, "test_interval": ti,
            "w": f32hex(res.w), "pulled": [f32hex(p) for p in res.pulled],
            "tests": [list(t) for t in res.tests], "accuracy_lines": res.accuracy_lines(),
            "model_rank0": oracle.format_model(res.pulled[0]),
        }
    with open(os.path.join(HERE, "trajectories.json"), "w") as f:
        json.dump(traj, f, indent=1)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
