"""Host logic of the product library (no GPU): the reference's parsing,
batching, init and model-format semantics, checked against the goldens
produced by the reference's own code (oracle/_ref) and against the oracle."""
from __future__ import annotations

import os

import numpy as np
import pytest

import distlr_amd as dlr
import oracle
from conftest import GOLDEN, read_golden_json
from parse_format import batches_text, csr_to_dense, parse_text_from_csr, sha
from test_oracle_golden import kat_rows


@pytest.mark.parametrize("row", list(kat_rows()), ids=lambda r: repr(r[0]))
def test_kat(row):
    s, iv, fb, nf, fields = row
    assert dlr.to_int(s) == iv
    assert dlr.to_float_bits(s) == fb
    assert dlr.split(s) == fields and len(fields) == nf


def test_parse_quirks_matches_reference():
    with open(os.path.join(GOLDEN, "quirks", "quirks.parse.txt")) as f:
        expect = f.read()
    ds = dlr.Dataset.load_libsvm(os.path.join(GOLDEN, "quirks", "quirks.libsvm"), 10)
    assert parse_text_from_csr(*ds.csr()) == expect


@pytest.mark.parametrize("nthreads", [1, 3, 16])
def test_parse_digests_match_reference(nthreads):
    g = read_golden_json("golden.json")
    for rel, meta in g["parse"].items():
        ds = dlr.Dataset.load_libsvm(os.path.join(GOLDEN, rel), meta["D"], nthreads=nthreads)
        assert sha(parse_text_from_csr(*ds.csr())) == meta["sha256"], rel


def test_parse_blank_lines_across_thread_chunks(tmp_path):
    # The blank-line quirk carries the previous token across lines; make the
    # file big enough that chunk boundaries land on blank lines.
    lines = []
    for i in range(40000):
        if i % 7 == 3:
            lines.append("")
        elif i % 11 == 5:
            lines.append("1")
        else:
            lines.append(f"{'+1' if i % 3 else '-1'} {1 + i % 9}:1 {10 + i % 5}:0.{i % 10000:04d}")
    p = tmp_path / "blank.libsvm"
    p.write_text("\n".join(lines) + "\n")
    X, y = oracle.load_dense(str(p), 20)
    for nt in (1, 2, 5, 8):
        ds = dlr.Dataset.load_libsvm(str(p), 20, nthreads=nt)
        rp, col, val, lab = ds.csr()
        assert np.array_equal(lab, y)
        assert np.array_equal(csr_to_dense(rp, col, val, 20).view(np.uint32), X.view(np.uint32))


def test_batches_match_reference():
    g = read_golden_json("golden.json")
    for key, meta in g["batches"].items():
        rel = key.split("@")[0]
        ds = dlr.Dataset.load_libsvm(os.path.join(GOLDEN, rel), meta["D"])
        rp, col, val, lab = ds.csr()
        X = csr_to_dense(rp, col, val, meta["D"])
        n, B = len(lab), meta["B"]
        assert dlr.num_batches(n, B) == meta["n_batches"]
        got = batches_text(X, lab, lambda b: dlr.batch_rows(n, B, b), meta["n_batches"])
        assert sha(got) == meta["sha256"], key


def test_batches_quirk_file():
    for B in (3, 5, -1, 25):
        with open(os.path.join(GOLDEN, "quirks", f"quirks.batches_B{B}.txt")) as f:
            expect = f.read()
        ds = dlr.Dataset.load_libsvm(os.path.join(GOLDEN, "quirks", "quirks.libsvm"), 10)
        rp, col, val, lab = ds.csr()
        X = csr_to_dense(rp, col, val, 10)
        n = len(lab)
        assert batches_text(X, lab, lambda b: dlr.batch_rows(n, B, b), dlr.num_batches(n, B)) == expect


def test_batch_edge_cases():
    assert dlr.num_batches(0, 10) == 0          # empty shard: no batches (reference: never terminates)
    assert dlr.num_batches(10, 0) < 0           # batch 0: rejected (reference: never terminates)
    assert dlr.num_batches(10, -1) == 1
    assert dlr.num_batches(10, 3) == 4
    assert list(dlr.batch_rows(10, 4, 2)) == [8, 9, 0, 1]
    assert list(dlr.batch_rows(3, 7, 0)) == [0, 1, 2, 0, 1, 2, 0]
    for n, B in [(10, 4), (7, 7), (5, 12), (1, 1), (100, 33)]:
        for b in range(dlr.num_batches(n, B)):
            assert np.array_equal(dlr.batch_rows(n, B, b), oracle.batch_rows(n, B, b))


def test_init_weight_matches_glibc():
    rk = read_golden_json("rand_kat.json")
    for seed, vals in rk.items():
        expect = np.array([np.float32(v) / np.float32(2147483647) for v in vals], dtype=np.float32)
        assert np.array_equal(dlr.init_weight(8, int(seed)).view(np.uint32), expect.view(np.uint32))
    for seed in (0, 3, 99):
        assert np.array_equal(dlr.init_weight(50000, seed).view(np.uint32),
                              oracle.init_weight(50000, seed).view(np.uint32))
    assert abs(float(dlr.init_weight(1)[0]) - 0.840187728) < 1e-9


def test_format_model_matches_oracle():
    w = np.concatenate([dlr.init_weight(200), np.array([1e-7, -2.5, 1.5e30, 0.0, 123456.7], np.float32)])
    assert dlr.format_model(w) == oracle.format_model(w)
    meta = read_golden_json("trajectories.json")["c1_W1_Bfull_mean"]
    pulled0 = np.frombuffer(bytes.fromhex(meta["pulled"][0]), dtype="<f4")
    assert dlr.format_model(pulled0) == meta["model_rank0"]


def test_key_ranges_partition():
    for D in (1, 7, 123, 1000, 1 << 20):
        for W in (1, 2, 3, 4, 8):
            ranges = [dlr.key_range(D, W, r) for r in range(W)]
            assert ranges[0][0] == 0 and ranges[-1][1] == D
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and a <= b
            chunk = (D + W - 1) // W
            assert all(b - a <= chunk for a, b in ranges)


def test_generator_deterministic_and_roundtrips(tmp_path):
    for vm in (0, 1):
        a = dlr.Dataset.generate(3000, 500, 17, value_mode=vm, seed=5, stream=2)
        b = dlr.Dataset.generate(3000, 500, 17, value_mode=vm, seed=5, stream=2, nthreads=3)
        for x, y in zip(a.csr(), b.csr()):
            assert np.array_equal(x, y)
        rp, col, val, lab = a.csr()
        assert np.all(np.diff(rp) == 17)
        for i in range(0, 3000, 97):
            c = col[rp[i]:rp[i + 1]]
            assert np.all(np.diff(c) > 0) and c.min() >= 0 and c.max() < 500
        p = str(tmp_path / f"g{vm}.libsvm")
        a.write_libsvm(p, vm)
        r = dlr.Dataset.load_libsvm(p, 500)
        for x, y in zip(a.csr(), r.csr()):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    c = dlr.Dataset.generate(3000, 500, 17, seed=5, stream=3)
    assert not np.array_equal(c.csr()[1], dlr.Dataset.generate(3000, 500, 17, seed=5, stream=2).csr()[1])


def test_generator_dense_rows():
    ds = dlr.Dataset.generate(50, 40, 40, value_mode=1, seed=1)
    rp, col, val, lab = ds.csr()
    assert np.all(np.diff(rp) == 40) and np.all(col.reshape(50, 40) == np.arange(40))


def test_parse_errors_are_loud(tmp_path):
    p = tmp_path / "bad.libsvm"
    p.write_text("+1 1:1 200:1\n")
    with pytest.raises(dlr.DLRError) as e:
        dlr.Dataset.load_libsvm(str(p), 10)
    assert e.value.code == -3 and ":1:" in str(e.value)
    p.write_text("+1 1:1\n-1 0:1\n")
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.load_libsvm(str(p), 10)
    p.write_text("+1 1:1\n-1 7\n")
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.load_libsvm(str(p), 10)
    with pytest.raises(dlr.DLRError) as e:
        dlr.Dataset.load_libsvm(str(tmp_path / "missing"), 10)
    assert e.value.code == -2


def test_from_csr_validation():
    ok = dlr.Dataset.from_csr([0, 2, 3], [1, 4, 0], [1, 2, 3], [1, 0], 5)
    assert ok.info() == (2, 3, 5)
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.from_csr([0, 2, 3], [4, 1, 0], [1, 2, 3], [1, 0], 5)   # unsorted
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.from_csr([0, 2, 3], [1, 5, 0], [1, 2, 3], [1, 0], 5)   # out of range
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.from_csr([0, 2, 3], [1, 4, 0], [1, 2, 3], [1, 2], 5)   # label not 0/1


def test_empty_file(tmp_path):
    p = tmp_path / "empty.libsvm"
    p.write_text("")
    ds = dlr.Dataset.load_libsvm(str(p), 4)
    assert ds.info() == (0, 0, 4)
