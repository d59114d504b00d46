"""cpu_baselines.py -- the two CPU baselines bench.py reports beside the GPU
numbers.  CPU BASELINES / TEST INFRASTRUCTURE
ONLY: imported by bench.py's cpu_baseline leg and tests/, never by the
product.

* reference_local_run / reference_inner_cost (build/liblr_refloop.so,
  ref_loop.cc): the reference's CPU path with its own cost structure --
  local.sh's W worker threads + in-process server, per-epoch re-parse into
  dense samples, lr.cc:35-39's O(B*D^2) loop with by-value feature copies.
  Its arithmetic is the oracle's, so its weights are bitwise the oracle's.
* omp_train_csr / omp_train_dense (build/liblr_cpu_omp.so, lr_cpu_omp.c):
  an efficient OpenMP trainer on the host's cores -- "build CPU path, not
  reference".
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
P = C.c_void_p
i64 = C.c_int64


def _load(name):
    path = os.path.join(HERE, "build", name)
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `make -C oracle`")
    return C.CDLL(path)


_ref = _load("liblr_refloop.so")
_ref.orc_ref_local_run.restype = C.c_int
_ref.orc_ref_local_run.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, P,
                                   C.POINTER(i64), C.POINTER(C.c_double), C.POINTER(i64), C.POINTER(i64)]
_ref.orc_ref_inner_cost.restype = C.c_double
_ref.orc_ref_inner_cost.argtypes = [C.c_int, C.c_int, i64]

_omp = _load("liblr_cpu_omp.so")
_omp.cpu_omp_threads.restype = C.c_int
_omp.cpu_omp_train_csr.restype = C.c_double
_omp.cpu_omp_train_csr.argtypes = [P, P, P, P, i64, i64, i64, P, C.c_float, C.c_float, i64, i64]
_omp.cpu_omp_train_dense.restype = C.c_double
_omp.cpu_omp_train_dense.argtypes = [P, P, i64, i64, i64, P, C.c_float, C.c_float, i64, i64]


def _p(a):
    return None if a is None else a.ctypes.data_as(P)


def reference_local_run(root: str, W: int, D: int, num_iteration: int, batch_size: int, test_interval: int,
                        lr: float, mode: int = 0):
    """Runs local.sh's job on DATA_DIR `root` with W worker threads.
    Returns (weights, sample_steps, seconds, last_correct, test_rows)."""
    w = np.zeros(D, np.float32)
    steps, sec, corr, rows = i64(), C.c_double(), i64(), i64()
    rc = _ref.orc_ref_local_run(root.encode(), W, D, num_iteration, batch_size, test_interval, lr, mode, _p(w),
                                C.byref(steps), C.byref(sec), C.byref(corr), C.byref(rows))
    if rc != 0:
        raise ValueError("orc_ref_local_run: bad argument")
    return w, steps.value, sec.value, corr.value, rows.value


def reference_inner_cost(D: int, n: int = 4, iters: int = 1000) -> float:
    """Seconds per (j, sample) iteration of lr.cc:35-39 at dimension D."""
    return float(_ref.orc_ref_inner_cost(D, n, iters))


def omp_threads() -> int:
    return int(_omp.cpu_omp_threads())


def omp_train_csr(row_ptr, col, val, label, D: int, B: int, w: np.ndarray, lr: float, C_: float = 1.0,
                  first_batch: int = 0, steps: int = 1) -> float:
    """In-place steps on w; val None = unit values.  Returns seconds."""
    el = _omp.cpu_omp_train_csr(_p(row_ptr), _p(col), _p(val), _p(label), len(label), D, B, _p(w), lr, C_,
                                first_batch, steps)
    if el < 0:
        raise ValueError("cpu_omp_train_csr failed")
    return el


def omp_train_dense(X, label, B: int, w: np.ndarray, lr: float, C_: float = 1.0, first_batch: int = 0,
                    steps: int = 1) -> float:
    el = _omp.cpu_omp_train_dense(_p(X), _p(label), X.shape[0], X.shape[1], B, _p(w), lr, C_, first_batch, steps)
    if el < 0:
        raise ValueError("cpu_omp_train_dense failed")
    return el
