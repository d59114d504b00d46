"""The N>1 data path on CPU through the LIBRARY's exchange code: world-size
2, 4 and 8 torch.distributed (gloo) runs of the engine's two exchange
protocols, checked bitwise against the oracle's multi-worker trajectories
(oracle.run_worker, main.cc:41-96 semantics), and the RCCL transport's own
calls for every rank (recorded, no GPU) checked to pair up.

What runs here is the engine's, not a restatement:
  * the step's collectives -- their kinds, sizes, offsets and order -- come
    from dlr_exchange_plan, the plan dlr_train_step itself issues
    (dist-lr_amd/csrc/dlr_exchange.h); gloo carries them between processes;
  * the server-side merge is dlr_merge_range / dlr_merge_touched: the
    kernels' own source (k_merge_update, k_sparse_merge, k_dense_l2) built
    for the host;
  * the key ranges are dlr_key_range's.
Only the per-rank pushed gradient comes from the oracle (the GPU kernels'
bitwise equivalent, tests/test_gpu_*): there is no GPU here.

  key range : ALL_TO_ALL of ceil(D/W)-key slices of every rank's pushed
              gradient -> rank-ordered merge of the owned range -> ALL_GATHER
              (or ALL_GATHER_PART per piece) of the merged ranges (the pull)
  touched   : ALL_GATHER of [count | cols | g] blocks (padded to the max
              touched count) -> every rank merges every touched column in
              rank order (non-touching ranks push the L2 term) and applies
              the L2-only update to the rest
"""
from __future__ import annotations

import os
import re
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from conftest import GOLDEN  # noqa: E402

D = 123
LR = 0.2
EPOCHS = 2
B = 64


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shards(world: int):
    """Rank r's training shard as CSR + dense (the oracle's form): the
    local.sh golden parts at W = 2, generated gen_data-shaped parts else."""
    import distlr_amd as dlr
    from parse_format import csr_to_dense
    out = []
    for r in range(world):
        if world == 2:
            ds = dlr.Dataset.load_libsvm(os.path.join(GOLDEN, "c1_tiny", "train", f"part-00{r + 1}"), D)
        else:
            ds = dlr.Dataset.generate(300, D, 14, value_mode=1, seed=7, stream=r + 1)  # (equal batch counts)
        rp, col, val, lab = ds.csr()
        out.append(((rp, col, val), lab, (csr_to_dense(rp, col, val, D), lab)))
    return out


def _worker(rank: int, world: int, port: int, protocol: str, mode: int, pieces: int, out: str):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    for p in (os.path.join(root, "dist-lr_amd"), os.path.join(root, "oracle"), os.path.dirname(__file__)):
        sys.path.insert(0, p)
    import distlr_amd as dlr
    import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    # (a rank that fails makes its peers' collectives time out, not hang)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        csr, lab, _ = _shards(world)[rank]
        N = len(lab)
        w = oracle.init_weight(D)
        kb, ke = dlr.key_range(D, world, rank)
        nb = oracle.num_batches(N, B)
        # every rank's batch size (the L2 term of its pushes), as gathered at load
        Bs = [None] * world
        dist.all_gather_object(Bs, B if B > 0 else N)
        ran = []  # the collectives this rank issued (kind, words, off, count)
        for it in range(EPOCHS):
            for b in range(nb):
                rows = oracle.batch_rows(N, B, b)
                g = oracle.grad_csr(csr, lab, rows, w)
                if protocol == "key_range":
                    plan = dlr.exchange_plan(dlr.EXCHANGE_KEY_RANGE, D, world, pieces)
                    (kind, chunk, _, _), pulls = plan[0], plan[1:]
                    assert kind == dlr.COLL_ALL_TO_ALL
                    send = np.zeros(chunk * world, np.float32)
                    send[:D] = g
                    recv = torch.zeros(chunk * world, dtype=torch.float32)
                    dist.all_to_all_single(recv, torch.from_numpy(send))
                    ran.append(plan[0])
                    full = np.zeros(chunk * world, np.float32)
                    full[:D] = w
                    own = full[rank * chunk:rank * chunk + (ke - kb)].copy()
                    dlr.merge_range(recv.numpy().reshape(world, chunk), own, LR, mode)  # rank-major
                    full[rank * chunk:rank * chunk + (ke - kb)] = own
                    for kind, words, off, count in pulls:
                        ran.append((kind, words, off, count))
                        if kind == dlr.COLL_ALL_GATHER:
                            parts = [torch.zeros(words, dtype=torch.float32) for _ in range(world)]
                            dist.all_gather(parts, torch.from_numpy(full[rank * words:(rank + 1) * words].copy()))
                            full = np.concatenate([t.numpy() for t in parts])
                        else:
                            assert kind == dlr.COLL_ALL_GATHER_PART
                            parts = [torch.zeros(count, dtype=torch.float32) for _ in range(world)]
                            mine = full[rank * words + off:rank * words + off + count].copy()
                            dist.all_gather(parts, torch.from_numpy(mine))
                            for q in range(world):
                                full[q * words + off:q * words + off + count] = parts[q].numpy()
                    w = full[:D].copy()
                else:
                    cols = np.unique(np.concatenate([csr[1][csr[0][r]:csr[0][r + 1]] for r in rows])).astype(np.int64)
                    cnt = torch.tensor([len(cols)], dtype=torch.int64)
                    dist.all_reduce(cnt, op=dist.ReduceOp.MAX)  # (the engine's touched cap, agreed at load)
                    cap = int(cnt.item())
                    plan = dlr.exchange_plan(dlr.EXCHANGE_TOUCHED, D, world, 0, cap)
                    assert len(plan) == 1 and plan[0][0] == dlr.COLL_ALL_GATHER and plan[0][1] == 1 + 2 * cap
                    blk = np.zeros(1 + 2 * cap, np.uint32)
                    blk[0] = len(cols)
                    blk[1:1 + len(cols)] = cols
                    blk[1 + cap:1 + cap + len(cols)] = g[cols].view(np.uint32)
                    blocks = [torch.zeros(1 + 2 * cap, dtype=torch.int32) for _ in range(world)]
                    dist.all_gather(blocks, torch.from_numpy(blk.view(np.int32)))
                    ran.append(plan[0])
                    lists = np.stack([t.numpy().view(np.uint32) for t in blocks])
                    dlr.merge_touched(lists, cap, Bs, w, LR, 1.0, mode)
        # all ranks issued the same collectives and hold the same replica
        allran = [None] * world
        dist.all_gather_object(allran, ran)
        assert all(r == allran[0] for r in allran), "ranks issued different collectives"
        allw = [torch.zeros(D, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(allw, torch.from_numpy(w))
        if rank == 0:
            np.save(out, np.stack([t.numpy() for t in allw]))
    finally:
        dist.destroy_process_group()


CASES = [(2, p, m, 0) for p in ("key_range", "touched") for m in (0, 1, 2)] + \
        [(2, "key_range", 0, 3), (4, "key_range", 0, 0), (4, "key_range", 2, 3), (4, "touched", 0, 0),
         (8, "key_range", 0, 16), (8, "key_range", 1, 0), (8, "touched", 2, 0)]


@pytest.mark.parametrize("world,protocol,mode,pieces", CASES)
def test_world_exchange_matches_oracle(tmp_path, world, protocol, mode, pieces):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import oracle
    out = str(tmp_path / "w.npy")
    mp.start_processes(_worker, args=(world, _free_port(), protocol, mode, pieces, out), nprocs=world, join=True,
                       start_method="spawn")
    ws = np.load(out)
    for r in range(1, world):
        assert np.array_equal(ws[0].view(np.uint32), ws[r].view(np.uint32)), f"replica {r} diverged"
    orc = oracle.run_worker([s[2] for s in _shards(world)], D, EPOCHS, B, LR, mode=mode)
    assert np.array_equal(ws[0].view(np.uint32), orc.w.view(np.uint32))


_LINE = re.compile(r"^(\w+)(?: uint32| int64)?(?: count=(\d+))?(?: (max|sum))?(?: peer=(\d+) at=(\d+))?$")


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("protocol,pieces", [("key_range", 0), ("key_range", 1), ("key_range", 3),
                                             ("key_range", 16), ("touched", 0)])
def test_rccl_calls_pair_up_across_ranks(world, protocol, pieces):
    # Every rank's RCCL calls for 3 steps (the RCCL transport recording its
    # calls instead of making them, dlr_rccl_trace): the same collectives
    # with the same counts on every rank, and inside every send/recv group
    # each ncclSend to q matched by q's ncclRecv from this rank, same count,
    # landing where the sender's block sits (at = sender * chunk + offset)
    import distlr_amd as dlr
    Dbig, cap = 1_000_003, 4321
    proto = dlr.EXCHANGE_KEY_RANGE if protocol == "key_range" else dlr.EXCHANGE_TOUCHED
    traces = [dlr.rccl_trace(proto, Dbig, world, r, pieces, cap, steps=3) for r in range(world)]
    chunk = -(-Dbig // world)
    plan = dlr.exchange_plan(proto, Dbig, world, pieces, cap)
    parsed = []
    for r, tr in enumerate(traces):
        assert tr, r
        ops = [m.groups() for m in map(_LINE.match, tr)]
        assert all(ops), tr
        parsed.append(ops)
    # the collectives (outside groups) agree on every rank, in order
    colls = [[(o[0], o[1]) for o in ops if o[0] in ("ncclAllToAll", "ncclAllGather", "ncclAllReduce")]
             for ops in parsed]
    assert all(c == colls[0] for c in colls)
    kinds = {dlr.COLL_ALL_TO_ALL: "ncclAllToAll", dlr.COLL_ALL_GATHER: "ncclAllGather"}
    assert colls[0] == [(kinds[k], str(words)) for k, words, _, _ in plan if k in kinds] * 3
    # the point-to-point groups pair up
    groups = []
    for r, ops in enumerate(parsed):
        gs, cur = [], None
        for name, count, _, peer, at in ops:
            if name == "ncclGroupStart":
                cur = []
            elif name == "ncclGroupEnd":
                gs.append(cur)
                cur = None
            elif name in ("ncclSend", "ncclRecv"):
                cur.append((name, int(count), int(peer), int(at)))
        groups.append(gs)
    nparts = sum(k == dlr.COLL_ALL_GATHER_PART for k, _, _, _ in plan)
    assert all(len(g) == 3 * nparts for g in groups)
    for gi in range(3 * nparts):
        for a in range(world):
            for name, count, peer, at in groups[a][gi]:
                if name != "ncclSend":
                    continue
                assert at // chunk == a  # the sender's own block
                match = [x for x in groups[peer][gi] if x == ("ncclRecv", count, a, at)]
                assert len(match) == 1, (gi, a, peer)
            peers = sorted(p for n, _, p, _ in groups[a][gi] if n == "ncclSend")
            assert peers == [q for q in range(world) if q != a]
