"""Drives the GPU engine (C-ABI) through RunWorker's semantics
(src/main.cc:124-170), so its results can be compared with
oracle.run_worker on the same inputs.

W == 1 runs the product's single-rank step (fused K2 -> K3+K4).
W > 1 on one GPU runs the parameter-server topology through the worker /
server entry points (dlr_worker_gradient / dlr_server_apply): one context
per worker plus a server context, all on device 0.  The RCCL exchange path
needs one GPU per rank and is exercised with a 1-rank communicator
(DLR_FORCE_COLLECTIVES=1) on the single-GPU box."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

import distlr_amd as dlr


@dataclass
class EngineRun:
    w: np.ndarray
    pulled: List[np.ndarray]
    tests: List[Tuple[int, int, int, float]] = field(default_factory=list)


def run_engine(shards: Sequence[dlr.Dataset], D: int, num_iteration: int, batch_size: int, learning_rate: float,
               test: Optional[dlr.Dataset] = None, test_interval: int = 10, mode: int = dlr.MODE_SYNC_MEAN,
               C_: float = 1.0, random_state: int = 0, dense: bool = False,
               order: int = dlr.ORDER_REFERENCE) -> EngineRun:
    """dense=True: the shards go through the dense path (K6, DataIter's own
    N x D layout) instead of the sparse one.  order: the engines' summation
    order (dlr_set_summation_order; the product default is the reference's)."""
    W = len(shards)
    w0 = dlr.init_weight(D, random_state)
    if dense:
        shards = [s if isinstance(s, dlr.DenseDataset) else dlr.DenseDataset.from_dataset(s) for s in shards]
        if test is not None and not isinstance(test, dlr.DenseDataset):
            test = dlr.DenseDataset.from_dataset(test)

    def load_train(eng, ds):
        return eng.load_train_dense(ds, batch_size) if dense else eng.load_train(ds, batch_size)

    def load_test(eng, ds):
        return eng.load_test_dense(ds) if dense else eng.load_test(ds)

    if W == 1:
        eng = dlr.Engine(D)
        try:
            eng.set_summation_order(order)
            eng.set_weights(w0)
            nb = load_train(eng, shards[0])
            if test is not None:
                load_test(eng, test)
            pulled = w0.copy()
            res = EngineRun(w=w0, pulled=[pulled])
            for it in range(num_iteration):
                for b in range(nb):
                    if it == num_iteration - 1 and b == nb - 1:
                        pulled = eng.get_weights()      # the last PullWeight_ of Train
                    eng.train_step(b, learning_rate, C_, mode)
                if test is not None and (it + 1) % test_interval == 0:
                    c, n, ll = eng.predict()
                    res.tests.append((it + 1, c, n, ll))
                    if it == num_iteration - 1:
                        pulled = eng.get_weights()  # Test pulled last
            res.w = eng.get_weights()
            res.pulled = [pulled]
            return res
        finally:
            eng.close()
    workers = [dlr.Engine(D) for _ in range(W)]
    server = dlr.Engine(D)
    try:
        for wk in workers:
            wk.set_summation_order(order)
        server.set_weights(w0)
        nbs = [load_train(wk, s) for wk, s in zip(workers, shards)]
        assert len(set(nbs)) == 1
        if test is not None:
            load_test(server, test)
        pulled = [w0.copy() for _ in range(W)]
        res = EngineRun(w=w0, pulled=pulled)
        for it in range(num_iteration):
            for b in range(nbs[0]):
                w = server.get_weights()
                grads = []
                for r, wk in enumerate(workers):
                    wk.set_weights(w)
                    pulled[r] = w
                    grads.append(wk.worker_gradient(b, C_))
                server.server_apply(grads, learning_rate, mode)
            if test is not None and (it + 1) % test_interval == 0:
                c, n, ll = server.predict()
                res.tests.append((it + 1, c, n, ll))
                pulled[0] = server.get_weights()
        res.w = server.get_weights()
        res.pulled = pulled
        return res
    finally:
        for e in workers + [server]:
            e.close()


def run_group(shards: Sequence, D: int, num_iteration: int, batch_size: int, learning_rate: float,
              test=None, test_interval: int = 10, mode: int = dlr.MODE_SYNC_MEAN, C_: float = 1.0,
              random_state: int = 0, dense: bool = False, device: int = 0, setup=None,
              order: int = dlr.ORDER_REFERENCE, preload=None) -> EngineRun:
    """RunWorker (main.cc:124-170) with W = len(shards) ranks of ONE device
    linked by the loopback transport (dlr_create_group): the product's
    world > 1 step -- key-range all-to-all, rank-ordered merge, in-place
    all-gather (or the touched-list exchange) -- with one host thread per
    rank, as bin/distlr drives its ranks."""
    import threading

    W = len(shards)
    w0 = dlr.init_weight(D, random_state)
    if dense:
        shards = [s if isinstance(s, dlr.DenseDataset) else dlr.DenseDataset.from_dataset(s) for s in shards]
        if test is not None and not isinstance(test, dlr.DenseDataset):
            test = dlr.DenseDataset.from_dataset(test)
    engines = dlr.Engine.create_group(D, W, device)
    pulled: List[Optional[np.ndarray]] = [None] * W
    finals: List[Optional[np.ndarray]] = [None] * W
    tests: List[Tuple[int, int, int, float]] = []
    errors: List[Optional[BaseException]] = [None] * W

    def rank_main(r: int):
        eng = engines[r]
        try:
            eng.set_summation_order(order)
            if preload is not None:
                preload(eng, r)
            eng.set_weights(w0)                      # every rank holds InitWeight_'s result (main.cc:141-148)
            nb = eng.load_train_dense(shards[r], batch_size) if dense else eng.load_train(shards[r], batch_size)
            if r == 0 and test is not None:
                eng.load_test_dense(test) if dense else eng.load_test(test)
            if setup is not None:
                setup(eng)
            p = w0.copy()
            for it in range(num_iteration):
                for b in range(nb):
                    if it == num_iteration - 1 and b == nb - 1:
                        p = eng.get_weights()        # the last PullWeight_ of Train (lr.cc:32)
                    eng.train_step(b, learning_rate, C_, mode)
                if r == 0 and test is not None and (it + 1) % test_interval == 0:
                    c, n, ll = eng.predict()
                    tests.append((it + 1, c, n, ll))
                    if it == num_iteration - 1:
                        p = eng.get_weights()
            pulled[r] = p
            finals[r] = eng.get_weights()
        except BaseException as e:  # noqa: BLE001 -- re-raised in the caller
            errors[r] = e
            eng.comm_abort(f"rank {r}: {e}")  # peers waiting in a collective fail now, not at the timeout

    try:
        th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        for e in engines:
            e.close()
    for e in errors:
        if e is not None:
            raise e
    for r in range(1, W):  # replicated weights: every rank ends with the same bits
        assert np.array_equal(finals[r].view(np.uint32), finals[0].view(np.uint32)), f"rank {r} weights differ"
    return EngineRun(w=finals[0], pulled=pulled, tests=tests)
