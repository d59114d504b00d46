"""Renders parse / batching results in oracle/_ref/ref_driver's text format,
so the oracle and the product can be compared with the reference-built
goldens (tests/golden/*.parse.txt and the sha256 digests in golden.json)."""
from __future__ import annotations

import hashlib

import numpy as np


def _bits(v) -> str:
    return "%08x" % int(np.float32(v).view(np.uint32))


def parse_text_from_csr(rp, col, val, label) -> str:
    out = [f"n {len(label)}"]
    for i in range(len(label)):
        a, b = int(rp[i]), int(rp[i + 1])
        items = " ".join(f"{int(col[k])}:{_bits(val[k])}" for k in range(a, b))
        out.append(f"{int(label[i])} {b - a}" + (" " + items if items else ""))
    return "\n".join(out) + "\n"


def parse_text_from_dense(X, y) -> str:
    out = [f"n {len(y)}"]
    for i in range(len(y)):
        nz = np.nonzero(X[i])[0]
        items = " ".join(f"{int(j)}:{_bits(X[i, j])}" for j in nz)
        out.append(f"{int(y[i])} {len(nz)}" + (" " + items if items else ""))
    return "\n".join(out) + "\n"


def _fnv_dense(x: np.ndarray) -> int:
    h = 1469598103934665603
    for byte in np.ascontiguousarray(x, dtype="<f4").tobytes():
        h ^= byte
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def batches_text(X, y, batch_rows_fn, n_batches: int) -> str:
    out = []
    for b in range(n_batches):
        rows = batch_rows_fn(b)
        out.append(f"batch {b} {len(rows)}")
        for r in rows:
            out.append("%d %016x" % (int(y[r]), _fnv_dense(X[r])))
    return "\n".join(out) + "\n"


def sha(text: str) -> str:
    return hashlib.sha256(text.encode("latin-1")).hexdigest()


def csr_to_dense(rp, col, val, D):
    n = len(rp) - 1
    X = np.zeros((n, D), dtype=np.float32)
    for i in range(n):
        X[i, col[rp[i]:rp[i + 1]]] = val[rp[i]:rp[i + 1]]
    return X
