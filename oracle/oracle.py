"""oracle.py -- TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU
restatement (oracle/lr_oracle.c -> oracle/build/liblr_oracle.so) and the
RunWorker orchestration of src/main.cc:124-170 built on it.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It is the checker, never the thing measured as the product.
See lr_oracle.c's header for what is pinned by the reference itself
(parsing: oracle/_ref + tests/golden) and what is a restatement
("parity unpinned" by reference execution: the LR arithmetic of lr.cc and
main.cc, whose build needs ps-lite's absent ps/ps.h).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liblr_oracle.so")
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built: run `make -C oracle`")
_lib = C.CDLL(LIB_PATH)
P = C.c_void_p
i64 = C.c_int64


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)


_sig("orc_to_int", C.c_int, C.c_char_p)
_sig("orc_to_float", C.c_float, C.c_char_p)
_sig("orc_split", C.c_int, C.c_char_p, C.c_char, C.c_char_p, C.c_int)
_sig("orc_parse_dense", C.c_long, C.c_char_p, C.c_int, P, P, C.c_long, C.POINTER(C.c_long))
_sig("orc_dense_to_csr", C.c_long, P, C.c_long, C.c_int, P, P, P, C.c_long)
_sig("orc_batch_rows", C.c_long, C.c_long, C.c_long, C.c_long, P)
_sig("orc_init_weight", None, C.c_int, P, C.c_long)
_sig("orc_grad_dense", None, P, P, C.c_int, P, C.c_long, P, C.c_float, P, P)
_sig("orc_grad_csr", None, P, P, P, P, C.c_long, P, C.c_long, P, C.c_float, P, P)
_sig("orc_server_update", None, P, P, C.c_int, C.c_long, C.c_float, C.c_int)
_sig("orc_predict_dense", None, P, P, C.c_long, C.c_int, P, P, P)
_sig("orc_predict_csr", None, P, P, P, P, C.c_long, P, P, P)
_sig("orc_accuracy", C.c_float, i64, C.c_long)
_sig("orc_format_model", C.c_long, P, C.c_long, C.c_char_p, C.c_long)

MODE_MEAN, MODE_LAST, MODE_ASYNC = 0, 1, 2


def _p(a):
    return a.ctypes.data_as(P)


def to_int(s: bytes | str) -> int:
    return _lib.orc_to_int(s.encode() if isinstance(s, str) else s)


def to_float(s: bytes | str) -> float:
    return _lib.orc_to_float(s.encode() if isinstance(s, str) else s)


def split(s: bytes | str, sep: str = ":") -> List[bytes]:
    b = s.encode() if isinstance(s, str) else s
    buf = C.create_string_buffer(2 * len(b) * (len(b) + 2) + 16)
    n = _lib.orc_split(b, sep.encode(), buf, len(buf))
    if n < 0:
        raise ValueError("split buffer too small")
    out, raw, pos = [], buf.raw, 0
    for _ in range(n):
        e = raw.index(b"\0", pos)
        out.append(raw[pos:e])
        pos = e + 1
    return out


class ParseError(ValueError):
    pass


def load_dense(path: str, D: int) -> Tuple[np.ndarray, np.ndarray]:
    """data_iter.h:16-35 -> (X float32 [n, D], y int32 [n])."""
    err = C.c_long(0)
    n = _lib.orc_parse_dense(path.encode(), D, None, None, 0, C.byref(err))
    if n < 0:
        raise ParseError(f"{path}: oracle parse error {n} at line {err.value}")
    X = np.zeros((n, D), dtype=np.float32)
    y = np.zeros(n, dtype=np.int32)
    m = _lib.orc_parse_dense(path.encode(), D, _p(X), _p(y), n, C.byref(err))
    if m != n:
        raise ParseError(f"{path}: oracle parse error {m}")
    return X, y


def dense_to_csr(X: np.ndarray):
    n, D = X.shape
    cap = int(np.count_nonzero(X))
    rp = np.zeros(n + 1, dtype=np.int64)
    col = np.zeros(max(cap, 1), dtype=np.int32)
    val = np.zeros(max(cap, 1), dtype=np.float32)
    k = _lib.orc_dense_to_csr(_p(np.ascontiguousarray(X)), n, D, _p(rp), _p(col), _p(val), cap)
    return rp, col[:k], val[:k]


def batch_rows(N: int, B: int, b: int) -> np.ndarray:
    Bn = N if B < 0 else B
    rows = np.zeros(Bn, dtype=np.int64)
    _lib.orc_batch_rows(N, B, b, _p(rows))
    return rows


def num_batches(N: int, B: int) -> int:
    return int(_lib.orc_batch_rows(N, B, 0, None))


def init_weight(D: int, random_state: int = 0) -> np.ndarray:
    w = np.zeros(D, dtype=np.float32)
    _lib.orc_init_weight(random_state, _p(w), D)
    return w


def grad_dense(X, y, rows, w, C_: float = 1.0) -> np.ndarray:
    D = X.shape[1]
    g = np.zeros(D, dtype=np.float32)
    scratch = np.zeros(len(rows), dtype=np.float32)
    _lib.orc_grad_dense(_p(X), _p(y), D, _p(rows), len(rows), _p(w), C_, _p(g), _p(scratch))
    return g


def grad_csr(csr, y, rows, w, C_: float = 1.0, return_resid: bool = False):
    """lr.cc:34-41 for one batch; with return_resid also the residuals
    sigma(z_s) - y_s per batch position s (lr.cc:36-37)."""
    rp, col, val = csr
    D = len(w)
    g = np.zeros(D, dtype=np.float32)
    scratch = np.zeros(len(rows), dtype=np.float32)
    _lib.orc_grad_csr(_p(rp), _p(col), _p(val), _p(y), D, _p(rows), len(rows), _p(w), C_, _p(g), _p(scratch))
    return (g, scratch) if return_resid else g


def server_update(w: np.ndarray, grads: Sequence[np.ndarray], lr: float, mode: int = MODE_MEAN) -> None:
    arr = (P * len(grads))(*[_p(g) for g in grads])
    _lib.orc_server_update(_p(w), arr, len(grads), len(w), lr, mode)


def predict_dense(X, y, w) -> Tuple[int, float]:
    c, ll = i64(0), C.c_double(0)
    _lib.orc_predict_dense(_p(X), _p(y), X.shape[0], X.shape[1], _p(w), C.byref(c), C.byref(ll))
    return c.value, ll.value


def predict_csr(csr, y, w) -> Tuple[int, float]:
    rp, col, val = csr
    c, ll = i64(0), C.c_double(0)
    _lib.orc_predict_csr(_p(rp), _p(col), _p(val), _p(y), len(y), _p(w), C.byref(c), C.byref(ll))
    return c.value, ll.value


def accuracy(correct: int, n: int) -> float:
    return float(_lib.orc_accuracy(correct, n))


def format_model(w: np.ndarray) -> str:
    w = np.ascontiguousarray(w, dtype=np.float32)
    need = _lib.orc_format_model(_p(w), len(w), None, 0)
    buf = C.create_string_buffer(need + 1)
    _lib.orc_format_model(_p(w), len(w), buf, need + 1)
    return buf.raw[:need].decode()


def format_g(x: float) -> str:
    """ostream default formatting of a float (%g, precision 6)."""
    return "%g" % float(np.float32(x))


@dataclass
class RunResult:
    w: np.ndarray                       # server weights after the last epoch
    pulled: List[np.ndarray]            # each worker's last-pulled weights (what SaveModel writes)
    tests: List[Tuple[int, int, int, float]] = field(default_factory=list)  # (iteration, correct, n, logloss)

    def accuracy_lines(self) -> List[str]:
        """lr.cc:59-62 without the HH:MM:SS prefix."""
        return [f"Iteration {it}, accuracy: {format_g(accuracy(c, n))}" for it, c, n, _ in self.tests]


def run_worker(shards: Sequence[Tuple[np.ndarray, np.ndarray]], D: int, num_iteration: int, batch_size: int,
               learning_rate: float, test: Optional[Tuple[np.ndarray, np.ndarray]] = None, test_interval: int = 10,
               mode: int = MODE_MEAN, C_: float = 1.0, random_state: int = 0, sparse: bool = True) -> RunResult:
    """main.cc:124-170 + lr.cc:28-63 with W = len(shards) workers.

    A shard is (X, y) with X dense (N x D) or, for huge D, the CSR tuple
    (row_ptr, col, val) that dense_to_csr would produce.

    Sync (modes MEAN/LAST): every worker pulls the same weights at step t
    (the server holds all pushes of a step until all W arrived), pushes
    arrive in rank order.  ASYNC: all workers pull the step's weights, the
    server applies their pushes one by one in rank order (the reference's
    async interleaving is timing-dependent; this fixes one order).
    Rank 0 tests after epoch i when (i+1) % test_interval == 0, after the
    epoch's last update (its last Push has returned)."""
    W = len(shards)
    w = init_weight(D, random_state)          # rank 0's initial push (main.cc:141-148)
    pulled = [w.copy() for _ in range(W)]
    Ns = [len(y) for _, y in shards]
    nbs = [num_batches(n, batch_size) for n in Ns]
    if len(set(nbs)) != 1:
        raise ValueError(f"workers have different batch counts {nbs}: the reference's sync merge mixes epochs")
    data = []
    for X, y in shards:
        if isinstance(X, tuple):        # already CSR (row_ptr, col, val): huge-D shards
            if not sparse:
                raise ValueError("CSR shards need sparse=True")
            data.append((X, y))
        else:
            data.append((dense_to_csr(X) if sparse else X, y))
    test_csr = (dense_to_csr(test[0]), test[1]) if (test is not None and sparse) else test
    res = RunResult(w=w, pulled=pulled)
    for it in range(num_iteration):
        for b in range(nbs[0]):
            grads = []
            for r in range(W):
                pulled[r] = w.copy()                        # PullWeight_ (lr.cc:32)
                Xr, yr = data[r]
                rows = batch_rows(Ns[r], batch_size, b)
                grads.append(grad_csr(Xr, yr, rows, pulled[r], C_) if sparse
                             else grad_dense(Xr, yr, rows, pulled[r], C_))
            server_update(w, grads, learning_rate, mode)    # PushGradient_ + DataHandle
        if test is not None and (it + 1) % test_interval == 0:
            pulled[0] = w.copy()                            # Test's PullWeight_ (lr.cc:48)
            if sparse:
                c, ll = predict_csr(test_csr[0], test_csr[1], pulled[0])
            else:
                c, ll = predict_dense(test[0], test[1], pulled[0])
            res.tests.append((it + 1, c, len(test[1]), ll))
    res.w = w
    res.pulled = pulled
    return res
