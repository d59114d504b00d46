"""Seeded synthetic DATA_DIR in the layout examples/gen_data.py writes
(gen_data.py:18-45): num_part train shards DATA_DIR/train/part-00{k}
(k = 1..num_part, part_size rows each), the test file DATA_DIR/test/part-001
and an empty DATA_DIR/models/ for LR::SaveModel.  The reference splits a
shuffled a9a download (unseeded) into those files; the a9a files are not
available offline, so the rows here come from the library's seeded
generator (dlr_dataset_generate: gen_data.py-shaped libsvm rows, planted
labels).  Train part k is row stream k, the test file
stream 1000, so a shard's content does not depend on num_part.

    python -m distlr_amd.gen_data --data-dir ./data --num-part 2 --rows 8140 \\
        --test-rows 16281 --features 123 --nnz 14 [--real] [--binary-cache]

--binary-cache also writes each file's binary CSR cache (<file>.dlrcsr,
Dataset.load_cached) so the first training run skips the text parse.
"""
from __future__ import annotations

import argparse
import os
import sys

import distlr_amd as dlr

TEST_STREAM = 1000


def generate(data_dir: str, num_part: int, rows: int, test_rows: int, features: int, nnz: int,
             real: bool = False, seed: int = 10, binary_cache: bool = False, hashed: bool = False) -> dict:
    """Writes the layout; returns {path: (rows, nnz)} of the files written."""
    vm = 1 if real else 0
    out = {}
    for sub in ("train", "test", "models"):
        os.makedirs(os.path.join(data_dir, sub), exist_ok=True)

    def make(n, stream):
        if hashed:
            return dlr.Dataset.generate_hashed(n, features, nnz, seed=seed, stream=stream)
        return dlr.Dataset.generate(n, features, nnz, value_mode=vm, seed=seed, stream=stream)

    jobs = [(os.path.join(data_dir, "train", f"part-00{k + 1}"), rows, k + 1) for k in range(num_part)]
    jobs.append((os.path.join(data_dir, "test", "part-001"), test_rows, TEST_STREAM))
    for path, n, stream in jobs:
        ds = make(n, stream)
        try:
            ds.write_libsvm(path, vm)
            if binary_cache:
                ds.save_binary(path + ".dlrcsr")
            out[path] = (ds.info()[0], ds.info()[1])
        finally:
            ds.free()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--data-dir", required=True)
    ap.add_argument("--num-part", type=int, default=4, help="train shards (gen_data.py num_part)")
    ap.add_argument("--rows", type=int, required=True, help="rows per train shard")
    ap.add_argument("--test-rows", type=int, required=True)
    ap.add_argument("--features", type=int, required=True)
    ap.add_argument("--nnz", type=int, required=True, help="non-zeros per row (fields when --hashed)")
    ap.add_argument("--real", action="store_true", help="4-decimal values in (0,1] instead of 1")
    ap.add_argument("--hashed", action="store_true", help="Criteo-shaped hashed Zipf fields (BASELINE C3)")
    ap.add_argument("--seed", type=int, default=10)
    ap.add_argument("--binary-cache", action="store_true")
    a = ap.parse_args(argv)
    if a.num_part < 1 or a.rows < 1 or a.test_rows < 1 or a.features < 1 or not 0 < a.nnz <= a.features:
        ap.error("sizes must be positive and nnz <= features")
    files = generate(a.data_dir, a.num_part, a.rows, a.test_rows, a.features, a.nnz, a.real, a.seed,
                     a.binary_cache, a.hashed)
    for path, (n, nnz) in files.items():
        print(f"{path}: {n} rows, {nnz} non-zeros")
    print("done.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
