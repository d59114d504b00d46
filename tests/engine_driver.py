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
               C_: float = 1.0, random_state: int = 0, dense: bool = False) -> EngineRun:
    """dense=True: the shards go through the dense path (K6, DataIter's own
    N x D layout) instead of the sparse one."""
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
