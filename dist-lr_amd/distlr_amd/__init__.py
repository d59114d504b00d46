"""ctypes binding of libdistlr_amd's C-ABI (include/distlr_amd.h).

The library is built in-tree (``make -C dist-lr_amd``) and loaded from
``dist-lr_amd/lib/libdistlr_amd.so``.  There is no fallback: if the library
is missing, importing this module raises.  Import ``torch`` (if at all)
BEFORE this module, so that the process has a single HIP runtime: the
library binds to whichever ``libamdhip64.so.7`` is already loaded.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
LIB_PATH = os.path.join(PKG, "lib", "libdistlr_amd.so")
# diagnostic tools only (tools/c2_stamps.py): a variant build of the same library
LIB_PATH = os.environ.get("DLR_LIB", LIB_PATH)

MODE_SYNC_MEAN = 0
MODE_SYNC_LAST = 1
MODE_ASYNC = 2
UNIQUE_ID_BYTES = 128
LAYOUT_CLASSIC, LAYOUT_LDS, LAYOUT_TOUCHED = 0, 1, 2
RESIDENCY_AUTO, RESIDENCY_DEVICE, RESIDENCY_STREAM = 0, 1, 2
STAGE_MARGIN, STAGE_GRADIENT, STAGE_UPDATE = 0, 1, 2
TRANSPORT_NONE, TRANSPORT_RCCL, TRANSPORT_LOOPBACK = 0, 1, 2
ORDER_REFERENCE, ORDER_FAST = 0, 1
E_DEVICE = -8  # an in-launch hand-off never came (dlr_sync)
# test-only producer faults (dlr_set_fault)
FAULT_NONE, FAULT_MG_PUBLISH, FAULT_REF_PUBLISH, FAULT_HOT_RING = 0, 1, 2, 3
# dlr_stage_counters indices
COUNT_HOT_CHAIN_LAUNCHES, COUNT_HOT_GIVEUPS, COUNT_COWAIT_SERIALISED, COUNT_MG_DEMOTED = 0, 1, 2, 3
COUNTERS = 4

# Exported symbols, in include/distlr_amd.h order (tests check the .so
# exports every one of them).
SYMBOLS = [
    "dlr_to_int", "dlr_to_float", "dlr_split",
    "dlr_dataset_load_libsvm", "dlr_dataset_from_csr", "dlr_dataset_generate", "dlr_dataset_generate_hashed",
    "dlr_dataset_write_libsvm", "dlr_dataset_save_binary", "dlr_dataset_load_binary", "dlr_dataset_info",
    "dlr_dataset_view", "dlr_dataset_free",
    "dlr_dense_from_dataset", "dlr_dense_from_array", "dlr_dense_generate", "dlr_dense_info", "dlr_dense_view",
    "dlr_dense_free",
    "dlr_num_batches", "dlr_batch_rows",
    "dlr_init_weight", "dlr_format_model", "dlr_key_range",
    "dlr_exchange_plan", "dlr_merge_range", "dlr_merge_touched", "dlr_rccl_trace",
    "dlr_get_unique_id", "dlr_create", "dlr_create_group", "dlr_comm_abort", "dlr_comm_info", "dlr_destroy", "dlr_last_error",
    "dlr_set_weights", "dlr_get_weights", "dlr_load_train", "dlr_load_test", "dlr_load_train_dense",
    "dlr_load_test_dense", "dlr_set_residency", "dlr_train_residency",
    "dlr_tuning_default", "dlr_tuning_from_env", "dlr_set_tuning", "dlr_get_tuning", "dlr_set_summation_order",
    "dlr_summation_order",
    "dlr_train_step", "dlr_train_epoch", "dlr_worker_gradient", "dlr_server_apply", "dlr_predict", "dlr_sync",
    "dlr_set_fault",
    "dlr_timing", "dlr_kernel_time", "dlr_stage_time", "dlr_stage_counters", "dlr_train_layout", "dlr_train_band_rows", "dlr_train_relabeled", "dlr_train_unit_values", "dlr_train_product_margin", "dlr_train_pm_strided", "dlr_train_hot_columns", "dlr_train_row_rounds",
    "dlr_set_exchange_overlap", "dlr_exchange_overlap", "dlr_set_exchange_pieces", "dlr_exchange_pieces",
    "dlr_memory_info", "dlr_stream_bytes",
]

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built: run `make -C dist-lr_amd` (or __graft_entry__.build())")

lib = C.CDLL(LIB_PATH)

i64 = C.c_int64
P = C.c_void_p


class GenSpec(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("num_feature_dim", C.c_int64),
        ("nnz_per_row", C.c_int32),
        ("value_mode", C.c_int32),
        ("seed", C.c_uint64),
        ("stream", C.c_uint64),
        ("positive_frac", C.c_double),
        ("label_noise", C.c_double),
        ("nthreads", C.c_int32),
    ]


class HashedSpec(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("num_feature_dim", C.c_int64),
        ("fields", C.c_int32),
        ("nthreads", C.c_int32),
        ("cardinality", C.c_int64),
        ("zipf_s", C.c_double),
        ("seed", C.c_uint64),
        ("stream", C.c_uint64),
        ("positive_frac", C.c_double),
        ("label_noise", C.c_double),
    ]


class DenseSpec(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("num_feature_dim", C.c_int64),
        ("seed", C.c_uint64),
        ("stream", C.c_uint64),
        ("positive_frac", C.c_double),
        ("label_noise", C.c_double),
        ("nthreads", C.c_int32),
        ("reserved", C.c_int32),
    ]


AUTO = -1  # DLR_AUTO: the engine's own choice


class Tuning(C.Structure):
    """dlr_tuning (include/distlr_amd.h): the loads' layout / kernel-form
    choices, every field AUTO or forced.  Tuning.from_env() is what a load
    uses unless Engine.set_tuning was called."""
    _fields_ = [(n, C.c_int64) for n in (
        "grad_layout", "product_margin", "pm_fused", "pm_in_gradient", "pm_split", "row_rounds",
        "band_rows", "band_pipeline", "band_hot", "hot_stream", "hot_stream_max", "margin_hot",
        "long_column", "long_piece", "long_sched",
        "relabel", "relabel_tail", "relabel_rare", "unit_values",
        "stream_coalesce", "stream_device_layout",
        "dense_grad", "dense_ref", "dense_ref_lead")]

    @classmethod
    def default(cls, **fields) -> "Tuning":
        t = cls()
        lib.dlr_tuning_default(C.byref(t))
        for k, v in fields.items():
            setattr(t, k, v)
        return t

    @classmethod
    def from_env(cls) -> "Tuning":
        t = cls()
        lib.dlr_tuning_from_env(C.byref(t))
        return t

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("dlr_to_int", C.c_int, C.c_char_p)
_sig("dlr_to_float", C.c_float, C.c_char_p)
_sig("dlr_split", C.c_int, C.c_char_p, C.c_char, C.c_char_p, C.c_int)
_sig("dlr_dataset_load_libsvm", C.c_int, C.c_char_p, i64, C.c_int, C.POINTER(P))
_sig("dlr_dataset_from_csr", C.c_int, i64, i64, P, P, P, P, C.POINTER(P))
_sig("dlr_dataset_generate", C.c_int, C.POINTER(GenSpec), C.POINTER(P))
_sig("dlr_dataset_generate_hashed", C.c_int, C.POINTER(HashedSpec), C.POINTER(P))
_sig("dlr_dense_from_dataset", C.c_int, P, C.POINTER(P))
_sig("dlr_dense_from_array", C.c_int, i64, i64, P, P, C.POINTER(P))
_sig("dlr_dense_generate", C.c_int, C.POINTER(DenseSpec), C.POINTER(P))
_sig("dlr_dense_info", C.c_int, P, C.POINTER(i64), C.POINTER(i64))
_sig("dlr_dense_view", C.c_int, P, C.POINTER(P), C.POINTER(P))
_sig("dlr_dense_free", None, P)
_sig("dlr_load_train_dense", C.c_int, P, P, i64, C.POINTER(i64))
_sig("dlr_load_test_dense", C.c_int, P, P)
_sig("dlr_set_residency", C.c_int, P, C.c_int)
_sig("dlr_train_residency", C.c_int, P)
_sig("dlr_set_summation_order", C.c_int, P, C.c_int)
_sig("dlr_summation_order", C.c_int, P)
_sig("dlr_dataset_write_libsvm", C.c_int, P, C.c_char_p, C.c_int)
_sig("dlr_dataset_save_binary", C.c_int, P, C.c_char_p)
_sig("dlr_dataset_load_binary", C.c_int, C.c_char_p, C.POINTER(P))
_sig("dlr_dataset_info", C.c_int, P, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64))
_sig("dlr_dataset_view", C.c_int, P, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P))
_sig("dlr_dataset_free", None, P)
_sig("dlr_num_batches", i64, i64, i64)
_sig("dlr_batch_rows", C.c_int, i64, i64, i64, P)
_sig("dlr_init_weight", C.c_int, C.c_int, P, i64)
_sig("dlr_format_model", C.c_int, P, i64, C.c_char_p, i64, C.POINTER(i64))
_sig("dlr_key_range", C.c_int, i64, C.c_int, C.c_int, C.POINTER(i64), C.POINTER(i64))
_sig("dlr_exchange_plan", C.c_int, C.c_int, i64, C.c_int, C.c_int, i64, C.POINTER(i64), C.c_int)
_sig("dlr_merge_range", C.c_int, P, C.c_int, i64, i64, P, C.c_float, C.c_int)
_sig("dlr_merge_touched", C.c_int, P, C.c_int, i64, P, P, i64, C.c_float, C.c_float, C.c_int)
_sig("dlr_rccl_trace", i64, C.c_int, i64, C.c_int, C.c_int, C.c_int, i64, C.c_int, C.c_char_p, i64)
_sig("dlr_get_unique_id", C.c_int, P)
_sig("dlr_create", C.c_int, C.c_int, C.c_int, C.c_int, P, i64, C.POINTER(P))
_sig("dlr_create_group", C.c_int, C.c_int, C.c_int, i64, P)
_sig("dlr_comm_abort", C.c_int, P, C.c_char_p)
_sig("dlr_comm_info", C.c_int, P, C.POINTER(C.c_int), C.POINTER(C.c_int))
_sig("dlr_destroy", None, P)
_sig("dlr_last_error", C.c_char_p, P)
_sig("dlr_set_weights", C.c_int, P, P, i64)
_sig("dlr_get_weights", C.c_int, P, P, i64)
_sig("dlr_load_train", C.c_int, P, P, i64, C.POINTER(i64))
_sig("dlr_load_test", C.c_int, P, P)
_sig("dlr_train_step", C.c_int, P, i64, C.c_float, C.c_float, C.c_int)
_sig("dlr_train_epoch", C.c_int, P, C.c_float, C.c_float, C.c_int)
_sig("dlr_worker_gradient", C.c_int, P, i64, C.c_float, P, i64)
_sig("dlr_server_apply", C.c_int, P, P, C.c_int, i64, C.c_float, C.c_int)
_sig("dlr_predict", C.c_int, P, C.POINTER(i64), C.POINTER(i64), C.POINTER(C.c_double))
_sig("dlr_sync", C.c_int, P)
_sig("dlr_set_fault", C.c_int, P, C.c_int)
_sig("dlr_tuning_default", None, P)
_sig("dlr_tuning_from_env", None, P)
_sig("dlr_set_tuning", C.c_int, P, P)
_sig("dlr_get_tuning", C.c_int, P, P)
_sig("dlr_timing", C.c_int, P, C.c_int)
_sig("dlr_kernel_time", C.c_int, P, C.c_int, C.POINTER(C.c_double), C.POINTER(i64))
_sig("dlr_stage_time", C.c_int, P, C.c_int, i64, i64, C.c_float, C.c_float, C.POINTER(C.c_double))
_sig("dlr_stage_counters", C.c_int, P, C.POINTER(i64), C.c_int)
_sig("dlr_train_layout", C.c_int, P)
_sig("dlr_train_band_rows", C.c_int, P)
_sig("dlr_train_relabeled", C.c_int, P)
_sig("dlr_train_unit_values", C.c_int, P)
_sig("dlr_train_product_margin", C.c_int, P)
_sig("dlr_train_pm_strided", C.c_int, P)
_sig("dlr_train_hot_columns", C.c_int, P)
_sig("dlr_train_row_rounds", C.c_int, P)
_sig("dlr_set_exchange_overlap", C.c_int, P, C.c_int)
_sig("dlr_exchange_overlap", C.c_int, P)
_sig("dlr_set_exchange_pieces", C.c_int, P, C.c_int)
_sig("dlr_exchange_pieces", C.c_int, P)
_sig("dlr_memory_info", C.c_int, P, C.POINTER(i64), C.POINTER(i64))
_sig("dlr_stream_bytes", C.c_int, P, C.POINTER(i64), C.POINTER(i64))


class DLRError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _check(rc: int, ctx=None):
    if rc < 0:
        msg = lib.dlr_last_error(ctx)
        raise DLRError(rc, msg.decode(errors="replace") if msg else "")
    return rc


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(P)


# ---------------------------------------------------------------- parsing

def to_int(s: str | bytes) -> int:
    return lib.dlr_to_int(s.encode() if isinstance(s, str) else s)


def to_float(s: str | bytes) -> float:
    return lib.dlr_to_float(s.encode() if isinstance(s, str) else s)


def to_float_bits(s: str | bytes) -> int:
    return int(np.float32(to_float(s)).view(np.uint32))


def split(s: str | bytes, sep: str = ":") -> list[bytes]:
    b = s.encode() if isinstance(s, str) else s
    buf = C.create_string_buffer(2 * len(b) * (len(b) + 2) + 16)
    n = _check(lib.dlr_split(b, sep.encode(), buf, len(buf)))
    out, raw, pos = [], buf.raw, 0
    for _ in range(n):
        e = raw.index(b"\0", pos)
        out.append(raw[pos:e])
        pos = e + 1
    return out


# ---------------------------------------------------------------- datasets

class Dataset:
    """A host CSR shard owned by the library (DataIter's storage)."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    @classmethod
    def load_libsvm(cls, path: str, num_feature_dim: int, nthreads: int = 0) -> "Dataset":
        h = P()
        _check(lib.dlr_dataset_load_libsvm(path.encode(), num_feature_dim, nthreads, C.byref(h)))
        return cls(h)

    @classmethod
    def from_csr(cls, row_ptr, col, val, label, num_feature_dim: int) -> "Dataset":
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        val = np.ascontiguousarray(val, dtype=np.float32)
        label = np.ascontiguousarray(label, dtype=np.int32)
        h = P()
        _check(lib.dlr_dataset_from_csr(len(row_ptr) - 1, num_feature_dim, _ptr(row_ptr), _ptr(col), _ptr(val),
                                        _ptr(label), C.byref(h)))
        return cls(h)

    @classmethod
    def generate(cls, n_rows: int, num_feature_dim: int, nnz_per_row: int, *, value_mode: int = 0,
                 seed: int = 10, stream: int = 0, positive_frac: float = 0.24, label_noise: float = 0.05,
                 nthreads: int = 0) -> "Dataset":
        spec = GenSpec(n_rows, num_feature_dim, nnz_per_row, value_mode, seed, stream, positive_frac,
                       label_noise, nthreads)
        h = P()
        _check(lib.dlr_dataset_generate(C.byref(spec), C.byref(h)))
        return cls(h)

    @classmethod
    def generate_hashed(cls, n_rows: int, num_feature_dim: int = 1 << 24, fields: int = 39, *,
                        cardinality: int = 1_000_000, zipf_s: float = 1.1, seed: int = 10, stream: int = 0,
                        positive_frac: float = 0.25, label_noise: float = 0.05, nthreads: int = 0) -> "Dataset":
        """Criteo-shaped hashed rows (BASELINE C3; dlr_dataset_generate_hashed)."""
        spec = HashedSpec(n_rows, num_feature_dim, fields, nthreads, cardinality, zipf_s, seed, stream,
                          positive_frac, label_noise)
        h = P()
        _check(lib.dlr_dataset_generate_hashed(C.byref(spec), C.byref(h)))
        return cls(h)

    def write_libsvm(self, path: str, value_mode: int = 0) -> None:
        _check(lib.dlr_dataset_write_libsvm(self._h, path.encode(), value_mode))

    def save_binary(self, path: str) -> None:
        """Binary CSR cache (dlr_dataset_save_binary)."""
        _check(lib.dlr_dataset_save_binary(self._h, path.encode()))

    @classmethod
    def load_binary(cls, path: str) -> "Dataset":
        h = P()
        _check(lib.dlr_dataset_load_binary(path.encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def load_cached(cls, path: str, num_feature_dim: int, nthreads: int = 0) -> "Dataset":
        """A libsvm shard through its binary cache `path + '.dlrcsr'`: parsed
        and cached on first use, reloaded while the cache is newer than the
        text and was written for the same D."""
        cache = path + ".dlrcsr"
        if os.path.exists(cache) and os.path.getmtime(cache) >= os.path.getmtime(path):
            try:
                ds = cls.load_binary(cache)
                if ds.info()[2] == num_feature_dim:
                    return ds
                ds.free()
            except DLRError:
                pass
        ds = cls.load_libsvm(path, num_feature_dim, nthreads)
        try:
            ds.save_binary(cache)
        except DLRError:
            pass  # a read-only data dir still trains from the text
        return ds

    def info(self) -> Tuple[int, int, int]:
        n, nnz, d = i64(), i64(), i64()
        _check(lib.dlr_dataset_info(self._h, C.byref(n), C.byref(nnz), C.byref(d)))
        return n.value, nnz.value, d.value

    @property
    def n_rows(self) -> int:
        return self.info()[0]

    def csr(self):
        """Copies of (row_ptr int64, col int32, val float32, label int32)."""
        n, nnz, _ = self.info()
        rp, cc, vv, ll = P(), P(), P(), P()
        _check(lib.dlr_dataset_view(self._h, C.byref(rp), C.byref(cc), C.byref(vv), C.byref(ll)))

        def arr(p, count, ctype, dtype):
            if count == 0:
                return np.zeros(0, dtype=dtype)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ctype)), shape=(count,)).astype(dtype, copy=True)

        return (arr(rp, n + 1, C.c_int64, np.int64), arr(cc, nnz, C.c_int32, np.int32),
                arr(vv, nnz, C.c_float, np.float32), arr(ll, n, C.c_int32, np.int32))

    def free(self):
        if self._h:
            lib.dlr_dataset_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DenseDataset:
    """Host dense shard (dlr_dense): row-major N x D fp32 + 0/1 labels."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    @classmethod
    def from_dataset(cls, ds: "Dataset") -> "DenseDataset":
        h = P()
        _check(lib.dlr_dense_from_dataset(ds.handle, C.byref(h)))
        return cls(h)

    @classmethod
    def from_array(cls, X: np.ndarray, label) -> "DenseDataset":
        X = np.ascontiguousarray(X, dtype=np.float32)
        y = np.ascontiguousarray(label, dtype=np.int32)
        h = P()
        _check(lib.dlr_dense_from_array(X.shape[0], X.shape[1], _ptr(X), _ptr(y), C.byref(h)))
        return cls(h)

    @classmethod
    def generate(cls, n_rows: int, num_feature_dim: int, *, seed: int = 10, stream: int = 0,
                 positive_frac: float = 0.3, label_noise: float = 0.05, nthreads: int = 0) -> "DenseDataset":
        spec = DenseSpec(n_rows, num_feature_dim, seed, stream, positive_frac, label_noise, nthreads, 0)
        h = P()
        _check(lib.dlr_dense_generate(C.byref(spec), C.byref(h)))
        return cls(h)

    def info(self) -> Tuple[int, int]:
        n, d = i64(), i64()
        _check(lib.dlr_dense_info(self._h, C.byref(n), C.byref(d)))
        return n.value, d.value

    def arrays(self):
        """(X, label) numpy views (valid while this object lives)."""
        n, d = self.info()
        xp, yp = P(), P()
        _check(lib.dlr_dense_view(self._h, C.byref(xp), C.byref(yp)))
        X = np.ctypeslib.as_array(C.cast(xp, C.POINTER(C.c_float)), shape=(n * d,)).reshape(n, d) if n else \
            np.zeros((0, d), np.float32)
        y = np.ctypeslib.as_array(C.cast(yp, C.POINTER(C.c_int32)), shape=(n,)) if n else np.zeros(0, np.int32)
        return X, y

    def free(self):
        if self._h:
            lib.dlr_dense_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def num_batches(n_rows: int, batch_size: int) -> int:
    return lib.dlr_num_batches(n_rows, batch_size)


def batch_rows(n_rows: int, batch_size: int, batch: int) -> np.ndarray:
    B = n_rows if batch_size < 0 else batch_size
    out = np.empty(B, dtype=np.int64)
    _check(lib.dlr_batch_rows(n_rows, batch_size, batch, _ptr(out)))
    return out


def init_weight(num_feature_dim: int, random_state: int = 0) -> np.ndarray:
    w = np.empty(num_feature_dim, dtype=np.float32)
    _check(lib.dlr_init_weight(random_state, _ptr(w), num_feature_dim))
    return w


def format_model(w: np.ndarray) -> str:
    w = np.ascontiguousarray(w, dtype=np.float32)
    need = i64()
    _check(lib.dlr_format_model(_ptr(w), len(w), None, 0, C.byref(need)))
    buf = C.create_string_buffer(need.value + 1)
    _check(lib.dlr_format_model(_ptr(w), len(w), buf, need.value + 1, C.byref(need)))
    return buf.raw[: need.value].decode()


def key_range(num_feature_dim: int, world: int, rank: int) -> Tuple[int, int]:
    b, e = i64(), i64()
    _check(lib.dlr_key_range(num_feature_dim, world, rank, C.byref(b), C.byref(e)))
    return b.value, e.value


EXCHANGE_KEY_RANGE, EXCHANGE_TOUCHED = 0, 1
COLL_ALL_TO_ALL, COLL_ALL_GATHER, COLL_ALL_GATHER_PART = 1, 2, 3


def exchange_plan(protocol: int, num_feature_dim: int, world: int, pieces: int = 0,
                  touched_cap: int = 0) -> List[Tuple[int, int, int, int]]:
    """The collectives of one world > 1 step, in order, on every rank:
    (kind, words, offset, count) each (dlr_exchange_plan)."""
    ops = (i64 * (4 * 64))()
    n = lib.dlr_exchange_plan(protocol, num_feature_dim, world, pieces, touched_cap, ops, 64)
    _check(min(n, 0))
    return [tuple(ops[4 * k:4 * k + 4]) for k in range(n)]


def merge_range(recv: np.ndarray, w_own: np.ndarray, lr: float, mode: int) -> None:
    """KVStoreDistServer::DataHandle on the owned keys, on the host, from the
    kernels' own source (dlr_merge_range): recv is (world, chunk) fp32,
    rank-major; w_own (n <= chunk) is updated in place."""
    recv = np.ascontiguousarray(recv, dtype=np.float32)
    assert w_own.dtype == np.float32 and w_own.flags.c_contiguous
    _check(lib.dlr_merge_range(_ptr(recv), recv.shape[0], recv.shape[1], w_own.shape[0], _ptr(w_own), lr, mode))


def merge_touched(lists: np.ndarray, cap: int, batch_rows, w: np.ndarray, lr: float, C_: float, mode: int) -> None:
    """The touched-list exchange's update of all D weights on the host
    (dlr_merge_touched): lists = (world, 1 + 2 * cap) uint32 blocks."""
    lists = np.ascontiguousarray(lists, dtype=np.uint32)
    br = np.ascontiguousarray(batch_rows, dtype=np.float32)
    assert w.dtype == np.float32 and w.flags.c_contiguous
    _check(lib.dlr_merge_touched(_ptr(lists), lists.shape[0], cap, _ptr(br), _ptr(w), w.shape[0], lr, C_, mode))


def rccl_trace(protocol: int, num_feature_dim: int, world: int, rank: int, pieces: int = 0,
               touched_cap: int = 0, steps: int = 1) -> List[str]:
    """The RCCL calls rank `rank` makes for `steps` steps, recorded instead
    of made (dlr_rccl_trace; no GPU)."""
    n = lib.dlr_rccl_trace(protocol, num_feature_dim, world, rank, pieces, touched_cap, steps, None, 0)
    _check(min(n, 0))
    buf = C.create_string_buffer(int(n))
    _check(min(lib.dlr_rccl_trace(protocol, num_feature_dim, world, rank, pieces, touched_cap, steps, buf, n), 0))
    return buf.value.decode().splitlines()


def get_unique_id() -> bytes:
    buf = C.create_string_buffer(UNIQUE_ID_BYTES)
    _check(lib.dlr_get_unique_id(buf))
    return buf.raw


# ---------------------------------------------------------------- engine

TIMER_MARGIN, TIMER_GRAD, TIMER_UPDATE, TIMER_EXCHANGE, TIMER_STEP = range(5)


class Engine:
    """One GPU context = one rank (dlr_ctx)."""

    def __init__(self, num_feature_dim: int, device: int = 0, rank: int = 0, world: int = 1,
                 unique_id: Optional[bytes] = None, _handle=None):
        self.D = num_feature_dim
        self.rank, self.world = rank, world
        if _handle is None:
            h = P()
            uid = C.create_string_buffer(unique_id, UNIQUE_ID_BYTES) if unique_id is not None else None
            _check(lib.dlr_create(device, rank, world, uid, num_feature_dim, C.byref(h)))
            _handle = h
        self._h = _handle
        self.n_batches = 0

    @classmethod
    def create_group(cls, num_feature_dim: int, world: int, device: int = 0) -> list:
        """`world` ranks on ONE device linked by the in-process loopback
        transport (dlr_create_group): the world > 1 engine path without
        RCCL.  Drive each engine from its own thread (collectives block until
        every rank arrives)."""
        hs = (P * world)()
        _check(lib.dlr_create_group(device, world, num_feature_dim, hs))
        return [cls(num_feature_dim, device, r, world, _handle=P(hs[r])) for r in range(world)]

    def comm_abort(self, why: str = "aborted") -> None:
        """This rank failed: release its peers' pending collectives
        (dlr_comm_abort)."""
        self._c(lib.dlr_comm_abort(self._h, why.encode()))

    def comm_info(self) -> Tuple[int, int]:
        """(ranks of the communicator, TRANSPORT_*) -- dlr_comm_info."""
        n, t = C.c_int(), C.c_int()
        self._c(lib.dlr_comm_info(self._h, C.byref(n), C.byref(t)))
        return n.value, t.value

    def _c(self, rc):
        return _check(rc, self._h)

    def set_weights(self, w: np.ndarray) -> None:
        w = np.ascontiguousarray(w, dtype=np.float32)
        self._c(lib.dlr_set_weights(self._h, _ptr(w), len(w)))

    def get_weights(self) -> np.ndarray:
        w = np.empty(self.D, dtype=np.float32)
        self._c(lib.dlr_get_weights(self._h, _ptr(w), self.D))
        return w

    def load_train(self, ds: Dataset, batch_size: int) -> int:
        nb = i64()
        self._c(lib.dlr_load_train(self._h, ds.handle, batch_size, C.byref(nb)))
        self.n_batches = nb.value
        return nb.value

    def load_test(self, ds: Dataset) -> None:
        self._c(lib.dlr_load_test(self._h, ds.handle))

    def load_train_dense(self, ds: DenseDataset, batch_size: int) -> int:
        nb = i64()
        self._c(lib.dlr_load_train_dense(self._h, ds.handle, batch_size, C.byref(nb)))
        self._train_src = ds  # a streamed shard reads the host rows in place: keep them alive
        return nb.value

    def set_tuning(self, tuning: "Tuning | None") -> None:
        """The tuning of this engine's later loads (None: the environment's
        at each load, the default; dlr_set_tuning)."""
        self._c(lib.dlr_set_tuning(self._h, C.byref(tuning) if tuning is not None else None))

    def get_tuning(self) -> "Tuning":
        t = Tuning()
        self._c(lib.dlr_get_tuning(self._h, C.byref(t)))
        return t

    def set_residency(self, mode: int) -> None:
        """RESIDENCY_AUTO / _DEVICE / _STREAM for the next dense training
        shard (dlr_set_residency)."""
        self._c(lib.dlr_set_residency(self._h, mode))

    def train_residency(self) -> int:
        rc = lib.dlr_train_residency(self._h)
        self._c(min(rc, 0))
        return rc

    def set_summation_order(self, order: int) -> None:
        """ORDER_REFERENCE (default: every sum in lr.cc's order, bitwise the
        reference's arithmetic) or ORDER_FAST (deterministic reordered long
        sums, within tolerance) for the next loaded training shard
        (dlr_set_summation_order)."""
        self._c(lib.dlr_set_summation_order(self._h, order))

    def summation_order(self) -> int:
        """The loaded training shard's order: ORDER_FAST only if some sum of
        it is actually reordered (dlr_summation_order)."""
        rc = lib.dlr_summation_order(self._h)
        self._c(min(rc, 0))
        return rc

    def load_test_dense(self, ds: DenseDataset) -> None:
        self._c(lib.dlr_load_test_dense(self._h, ds.handle))

    def train_step(self, batch: int, lr: float, C_: float = 1.0, mode: int = MODE_SYNC_MEAN) -> None:
        self._c(lib.dlr_train_step(self._h, batch, lr, C_, mode))

    def train_epoch(self, lr: float, C_: float = 1.0, mode: int = MODE_SYNC_MEAN) -> None:
        self._c(lib.dlr_train_epoch(self._h, lr, C_, mode))

    def worker_gradient(self, batch: int, C_: float = 1.0) -> np.ndarray:
        g = np.empty(self.D, dtype=np.float32)
        self._c(lib.dlr_worker_gradient(self._h, batch, C_, _ptr(g), self.D))
        return g

    def server_apply(self, grads, lr: float, mode: int = MODE_SYNC_MEAN) -> None:
        G = np.ascontiguousarray(np.stack(grads) if isinstance(grads, (list, tuple)) else grads, dtype=np.float32)
        assert G.ndim == 2 and G.shape[1] == self.D
        self._c(lib.dlr_server_apply(self._h, _ptr(G), G.shape[0], self.D, lr, mode))

    def predict(self) -> Tuple[int, int, float]:
        c, n, ll = i64(), i64(), C.c_double()
        self._c(lib.dlr_predict(self._h, C.byref(c), C.byref(n), C.byref(ll)))
        return c.value, n.value, ll.value

    def sync(self) -> None:
        self._c(lib.dlr_sync(self._h))

    def set_fault(self, fault: int) -> None:
        """TEST ONLY: withhold one in-launch producer (FAULT_*) in the next
        steps; they must then raise DLRError(E_DEVICE) (dlr_set_fault)."""
        self._c(lib.dlr_set_fault(self._h, fault))

    def timing(self, enable: bool) -> None:
        self._c(lib.dlr_timing(self._h, 1 if enable else 0))

    def kernel_time(self, which: int) -> Tuple[float, int]:
        ms, n = C.c_double(), i64()
        self._c(lib.dlr_kernel_time(self._h, which, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def stage_time(self, stage: int, first_batch: int, count: int, lr: float = 0.2, C_: float = 1.0) -> float:
        """Average ms of one kernel stage over `count` consecutive launches
        between one event pair (dlr_stage_time)."""
        ms = C.c_double()
        self._c(lib.dlr_stage_time(self._h, stage, first_batch, count, lr, C_, C.byref(ms)))
        return ms.value

    def stage_counters(self) -> dict:
        """Event counts since the shard was loaded (dlr_stage_counters):
        hot_chain_launches, hot_giveups, cowait_serialised, mg_demoted."""
        out = (i64 * COUNTERS)()
        self._c(lib.dlr_stage_counters(self._h, out, COUNTERS))
        return {"hot_chain_launches": out[COUNT_HOT_CHAIN_LAUNCHES], "hot_giveups": out[COUNT_HOT_GIVEUPS],
                "cowait_serialised": out[COUNT_COWAIT_SERIALISED], "mg_demoted": out[COUNT_MG_DEMOTED]}

    def train_layout(self) -> int:
        """LAYOUT_CLASSIC / LAYOUT_LDS / LAYOUT_TOUCHED of the loaded shard."""
        rc = lib.dlr_train_layout(self._h)
        self._c(min(rc, 0))
        return rc

    def train_band_rows(self) -> int:
        """Rows per band when the classic layout's short columns are summed
        in row bands (large batches), else 0 (dlr_train_band_rows)."""
        rc = lib.dlr_train_band_rows(self._h)
        self._c(min(rc, 0))
        return rc

    def train_relabeled(self) -> bool:
        """Whether the loaded sparse shard's columns are in frequency order
        (dlr_train_relabeled)."""
        rc = lib.dlr_train_relabeled(self._h)
        self._c(min(rc, 0))
        return rc == 1

    def train_unit_values(self) -> bool:
        """Whether the loaded sparse shard is unit-valued (every value 1.0f):
        no value arrays are stored and the UNIT kernels run
        (dlr_train_unit_values)."""
        rc = lib.dlr_train_unit_values(self._h)
        self._c(min(rc, 0))
        return rc == 1

    def train_hot_columns(self) -> int:
        """Hot columns whose chains run from the product stream (one
        k_hot_chain launch per step), 0 = per-band k_band_hot or none
        (dlr_train_hot_columns)."""
        rc = lib.dlr_train_hot_columns(self._h)
        self._c(min(rc, 0))
        return rc

    def train_product_margin(self) -> int:
        """0: gather margin; 1: product margin with a separate pass 1; 2:
        product margin with pass 1 fused into the previous step's gradient
        (dlr_train_product_margin)."""
        rc = lib.dlr_train_product_margin(self._h)
        self._c(min(rc, 0))
        return rc

    def train_pm_strided(self) -> int:
        """1: every batch's product-margin regions at fixed strides; 0: none
        (packed, or no product margin); 2: some (dlr_train_pm_strided)."""
        rc = lib.dlr_train_pm_strided(self._h)
        self._c(min(rc, 0))
        return rc

    def train_row_rounds(self) -> int:
        """Rounds of the row-round gradient (k_grad_rt), 0 for k_grad_lds or
        another layout (dlr_train_row_rounds)."""
        rc = lib.dlr_train_row_rounds(self._h)
        self._c(min(rc, 0))
        return rc

    def set_exchange_overlap(self, on: bool) -> None:
        """World > 1, product margin: all-gather in pieces overlapped with
        the next batch's pass 1 (dlr_set_exchange_overlap; default on)."""
        self._c(lib.dlr_set_exchange_overlap(self._h, 1 if on else 0))

    def exchange_overlap(self) -> bool:
        rc = lib.dlr_exchange_overlap(self._h)
        self._c(min(rc, 0))
        return rc == 1

    def set_exchange_pieces(self, pieces: int) -> None:
        """Pieces of the overlapped all-gather (1..16, default 4) for the
        next load_train (dlr_set_exchange_pieces; the ranks must agree)."""
        self._c(lib.dlr_set_exchange_pieces(self._h, int(pieces)))

    def exchange_pieces(self) -> int:
        """The loaded shard's piece count (0: the gather is not pieced)."""
        rc = lib.dlr_exchange_pieces(self._h)
        self._c(min(rc, 0))
        return rc

    def memory_info(self) -> Tuple[int, int]:
        a, b = i64(), i64()
        self._c(lib.dlr_memory_info(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def stream_bytes(self) -> Tuple[int, int]:
        """(mean, max) host->device bytes staged per batch of a streamed
        training shard (dlr_stream_bytes); (0, 0) when resident."""
        a, b = i64(), i64()
        self._c(lib.dlr_stream_bytes(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def close(self) -> None:
        if self._h:
            lib.dlr_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
