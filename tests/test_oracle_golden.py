"""Pins the oracle (oracle/lr_oracle.c) before it is trusted as the checker.

Parsing and batching are checked against outputs of the reference's own
util.cc + data_iter.h (oracle/_ref, captured in tests/golden/ by
make_golden.py); weight init against glibc's rand; the LR arithmetic
restatement against its frozen trajectories (parity unpinned by reference
execution -- lr.cc/main.cc need ps-lite, absent) and against its own dense
form (sparse port == dense restatement, bitwise)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, read_golden_json
from parse_format import batches_text, parse_text_from_dense, sha


def kat_rows():
    with open(os.path.join(GOLDEN, "kat_strings.txt"), "rb") as f:
        strings = f.read().split(b"\n")[:-1]
    with open(os.path.join(GOLDEN, "kat.tsv"), "rb") as f:
        rows = f.read().split(b"\n")[:-1]
    assert len(strings) == len(rows)
    for s, r in zip(strings, rows):
        head, *fields = r.split(b"\t")
        iv, fb, nf = head.split(b" ")
        yield s, int(iv), int(fb, 16), int(nf), [bytes.fromhex(x.decode()) for x in fields]


@pytest.mark.parametrize("row", list(kat_rows()), ids=lambda r: repr(r[0]))
def test_oracle_kat(row):
    s, iv, fb, nf, fields = row
    assert oracle.to_int(s) == iv
    assert int(np.float32(oracle.to_float(s)).view(np.uint32)) == fb
    assert oracle.split(s) == fields and len(fields) == nf


def test_survey_known_answers():
    # SURVEY.md 4.4 known answers, re-derived from util.cc by oracle/_ref.
    assert np.float32(oracle.to_float("0.333333")) == np.float32(0.333333015)
    assert oracle.to_float("-0.5") == -29.5
    assert oracle.to_float("1e-3") == 6273.0
    assert oracle.to_int("1.0") == 80
    assert oracle.split("a:b:c:d") == [b"a", b"b:c", b"c:d", b"d"]


def test_oracle_parse_quirks():
    with open(os.path.join(GOLDEN, "quirks", "quirks.parse.txt")) as f:
        expect = f.read()
    X, y = oracle.load_dense(os.path.join(GOLDEN, "quirks", "quirks.libsvm"), 10)
    assert parse_text_from_dense(X, y) == expect


@pytest.mark.parametrize("B", [3, 5, -1, 25])
def test_oracle_batches_quirks(B):
    with open(os.path.join(GOLDEN, "quirks", f"quirks.batches_B{B}.txt")) as f:
        expect = f.read()
    X, y = oracle.load_dense(os.path.join(GOLDEN, "quirks", "quirks.libsvm"), 10)
    n = len(y)
    got = batches_text(X, y, lambda b: oracle.batch_rows(n, B, b), oracle.num_batches(n, B))
    assert got == expect


def test_oracle_parse_digests():
    g = read_golden_json("golden.json")
    for rel, meta in g["parse"].items():
        X, y = oracle.load_dense(os.path.join(GOLDEN, rel), meta["D"])
        assert len(y) == meta["n"]
        assert sha(parse_text_from_dense(X, y)) == meta["sha256"], rel


def test_oracle_batch_digests():
    g = read_golden_json("golden.json")
    for key, meta in g["batches"].items():
        rel = key.split("@")[0]
        X, y = oracle.load_dense(os.path.join(GOLDEN, rel), meta["D"])
        n, B = len(y), meta["B"]
        assert oracle.num_batches(n, B) == meta["n_batches"]
        got = batches_text(X, y, lambda b: oracle.batch_rows(n, B, b), meta["n_batches"])
        assert sha(got) == meta["sha256"], key


def test_oracle_rand_kat():
    rk = read_golden_json("rand_kat.json")
    for seed, vals in rk.items():
        w = oracle.init_weight(8, int(seed))
        expect = np.array([np.float32(v) / np.float32(2147483647) for v in vals], dtype=np.float32)
        assert np.array_equal(w.view(np.uint32), expect.view(np.uint32))
    assert rk["0"][0] == 1804289383 and rk["0"] == rk["1"]   # glibc: srand(0) == srand(1)


def _load_shards(meta):
    base = os.path.join(GOLDEN, meta["dataset"])
    D = meta["D"]
    shards = [oracle.load_dense(os.path.join(base, "train", f"part-00{p + 1}"), D) for p in range(meta["workers"])]
    test = oracle.load_dense(os.path.join(base, "test", "part-001"), D)
    return shards, test


@pytest.mark.parametrize("name", list(read_golden_json("trajectories.json").keys()))
def test_oracle_trajectories_frozen(name):
    meta = read_golden_json("trajectories.json")[name]
    shards, test = _load_shards(meta)
    for sparse in (True, False):
        res = oracle.run_worker(shards, meta["D"], meta["num_iteration"], meta["batch_size"], meta["learning_rate"],
                                test=test, test_interval=meta["test_interval"], mode=meta["mode"], sparse=sparse)
        assert res.w.astype("<f4").tobytes().hex() == meta["w"]
        assert [p.astype("<f4").tobytes().hex() for p in res.pulled] == meta["pulled"]
        assert res.accuracy_lines() == meta["accuracy_lines"]
        assert oracle.format_model(res.pulled[0]) == meta["model_rank0"]


def test_oracle_modes_agree_at_one_worker():
    meta = read_golden_json("trajectories.json")["c1_W1_B7_mean"]
    shards, test = _load_shards(meta)
    ws = []
    for mode in (oracle.MODE_MEAN, oracle.MODE_LAST, oracle.MODE_ASYNC):
        res = oracle.run_worker(shards, meta["D"], 1, 7, 0.2, mode=mode)
        ws.append(res.w.view(np.uint32))
    assert np.array_equal(ws[0], ws[1]) and np.array_equal(ws[0], ws[2])


def test_oracle_model_format_matches_ostream():
    # lr.cc:75-79: "D\n", "%g " per weight, "\n"
    w = np.array([0.840187728, 1e-7, -2.5, 123456789.0, 0.0], dtype=np.float32)
    assert oracle.format_model(w) == "5\n0.840188 1e-07 -2.5 1.23457e+08 0 \n"
