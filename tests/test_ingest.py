"""Ingest: the binary CSR cache round trip and its
integrity checks, and the gen_data.py-layout generator (gen_data.py:18-45)
whose text files reparse bitwise to the generated shards."""
from __future__ import annotations

import os

import numpy as np
import pytest

import distlr_amd as dlr
from distlr_amd import gen_data


def csr(ds):
    rp, col, val, lab = ds.csr()
    return [np.array(a) for a in (rp, col, val, lab)]


def same(a, b):
    for x, y in zip(csr(a), csr(b)):
        assert x.dtype == y.dtype and x.tobytes() == y.tobytes()


@pytest.mark.parametrize("value_mode", [0, 1])
def test_binary_cache_round_trip(tmp_path, value_mode):
    ds = dlr.Dataset.generate(777, 1000, 13, value_mode=value_mode, seed=3, stream=2)
    p = str(tmp_path / "shard.dlrcsr")
    ds.save_binary(p)
    back = dlr.Dataset.load_binary(p)
    assert back.info() == ds.info()
    same(back, ds)


def test_binary_cache_empty_rows(tmp_path):
    rp = np.array([0, 0, 2, 2, 3], np.int64)
    ds = dlr.Dataset.from_csr(rp, np.array([1, 5, 0], np.int32), np.array([1.5, 2.0, 3.0], np.float32),
                              np.array([0, 1, 1, 0], np.int32), 6)
    p = str(tmp_path / "e.dlrcsr")
    ds.save_binary(p)
    same(dlr.Dataset.load_binary(p), ds)


def test_binary_cache_rejects_damage(tmp_path):
    ds = dlr.Dataset.generate(200, 50, 5, value_mode=1, seed=4, stream=1)
    p = str(tmp_path / "d.dlrcsr")
    ds.save_binary(p)
    raw = bytearray(open(p, "rb").read())
    flipped = bytearray(raw)
    flipped[len(raw) // 2] ^= 0x40                     # one bit in the arrays
    open(str(tmp_path / "flip.dlrcsr"), "wb").write(flipped)
    with pytest.raises(dlr.DLRError, match="checksum"):
        dlr.Dataset.load_binary(str(tmp_path / "flip.dlrcsr"))
    open(str(tmp_path / "short.dlrcsr"), "wb").write(raw[:-4])
    with pytest.raises(dlr.DLRError, match="size"):
        dlr.Dataset.load_binary(str(tmp_path / "short.dlrcsr"))
    open(str(tmp_path / "text.dlrcsr"), "wb").write(b"+1 3:1\n")
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.load_binary(str(tmp_path / "text.dlrcsr"))
    with pytest.raises(dlr.DLRError):
        dlr.Dataset.load_binary(str(tmp_path / "missing.dlrcsr"))


def test_load_cached_parses_once(tmp_path):
    ds = dlr.Dataset.generate(300, 123, 14, value_mode=1, seed=5, stream=1)
    txt = str(tmp_path / "part-001")
    ds.write_libsvm(txt, 1)
    first = dlr.Dataset.load_cached(txt, 123)
    assert os.path.exists(txt + ".dlrcsr")
    same(first, dlr.Dataset.load_libsvm(txt, 123))
    os.utime(txt + ".dlrcsr", (os.path.getmtime(txt) + 10,) * 2)
    same(dlr.Dataset.load_cached(txt, 123), first)
    # a cache written for another D is not used
    dlr.Dataset.generate(10, 77, 3, seed=1).save_binary(txt + ".dlrcsr")
    os.utime(txt + ".dlrcsr", (os.path.getmtime(txt) + 20,) * 2)
    same(dlr.Dataset.load_cached(txt, 123), first)


@pytest.mark.parametrize("real,hashed", [(False, False), (True, False), (False, True)])
def test_gen_data_layout(tmp_path, real, hashed):
    d = str(tmp_path / "data")
    D = 4096 if hashed else 123
    rc = gen_data.main(["--data-dir", d, "--num-part", "2", "--rows", "500", "--test-rows", "321",
                        "--features", str(D), "--nnz", "14", "--binary-cache"] + (["--real"] if real else [])
                       + (["--hashed"] if hashed else []))
    assert rc == 0
    assert sorted(os.listdir(os.path.join(d, "train"))) == ["part-001", "part-001.dlrcsr", "part-002",
                                                          "part-002.dlrcsr"]
    assert os.path.isdir(os.path.join(d, "models"))
    for k in (1, 2):
        path = os.path.join(d, "train", f"part-00{k}")
        parsed = dlr.Dataset.load_libsvm(path, D)
        same(parsed, dlr.Dataset.load_binary(path + ".dlrcsr"))
        assert parsed.info()[0] == 500
        if hashed:
            gen = dlr.Dataset.generate_hashed(500, D, 14, seed=10, stream=k)
        else:
            gen = dlr.Dataset.generate(500, D, 14, value_mode=1 if real else 0, seed=10, stream=k)
        same(parsed, gen)  # text round trip is bitwise (ToFloat-exact values)
    test = dlr.Dataset.load_libsvm(os.path.join(d, "test", "part-001"), D)
    assert test.info()[0] == 321
