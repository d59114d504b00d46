#!/usr/bin/env python3
"""bench.py -- whole-node training throughput of the dist-lr hot path.

Workload (BASELINE.json configs[1], "C2"): synthetic sparse LR, 10M samples
x 1M features, 50 distinct uniform columns per row, 4-decimal values in
(0,1] (gen_data.py-shaped, seeded), batch 65,536 rows, sync SGD lr 0.2,
C = 1.  One step = one LR::Train batch: margin + sigmoid + residual, Xᵀr
gradient + L2, (exchange), SGD update.  Weak scaling: every rank trains its
own 10M-row shard (rank r = part-00{r+1}, like main.cc:158).

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: launched by torch.distributed.run, one process per GPU.)

Prints ONE JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

try:
    import torch  # noqa: F401  -- loaded first: the library binds to torch's HIP runtime
    import torch.distributed as dist
except Exception:  # pragma: no cover
    torch = None
    dist = None

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dist-lr_amd"))

import distlr_amd as dlr  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--rows", type=int, default=10_000_000, help="training rows per GPU shard")
    ap.add_argument("--features", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=50)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--lr", type=float, default=0.2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per step (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def alg_bytes_per_step(B: int, nnz: int, D: int) -> int:
    """8*nnz + 8 bytes per sample (int32 col + fp32 val per
    nnz; row offset + label per row) + 8*D/B per sample (dense-L2 weight
    read + write), times the B samples of one step."""
    return B * (8 * nnz + 8) + 8 * D


def cpu_baseline(args, D: int) -> dict:
    """The oracle's sparse port (oracle/lr_oracle.c, bitwise equal to the
    reference arithmetic) on host cores, same batch shape; a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker only: timed as the CPU baseline, never as the product

    B = args.batch
    n_rows = 4 * B
    ds = dlr.Dataset.generate(n_rows, D, args.nnz, value_mode=1, seed=10, stream=1)
    rp, col, val, lab = ds.csr()
    w = dlr.init_weight(D)
    rows = [oracle.batch_rows(n_rows, B, b) for b in range(4)]
    done, t0 = 0, time.perf_counter()
    while True:
        g = oracle.grad_csr((rp, col, val), lab, rows[done % 4], w)
        oracle.server_update(w, [g], args.lr)
        done += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or done >= 5000:
            break
    return {"value": round(done * B / el, 1), "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": f"{done} steps of B={B}, D={D}, {args.nnz} nnz/row (oracle sparse port, 1 thread) in "
                      f"{el:.1f} s"}


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus N > 1 needs torch.distributed.run (one process per GPU)")
    distributed = world > 1
    if distributed:
        dist.init_process_group("gloo")   # control plane only; data path is RCCL inside the library
    D, B = args.features, args.batch

    uid = None
    if distributed:
        obj = [dlr.get_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]

    t_setup = time.perf_counter()
    ds = dlr.Dataset.generate(args.rows, D, args.nnz, value_mode=1, seed=10, stream=rank + 1)
    t_gen = time.perf_counter() - t_setup
    eng = dlr.Engine(D, device=local, rank=rank, world=world, unique_id=uid)
    eng.set_weights(dlr.init_weight(D))
    nb = eng.load_train(ds, B)
    train_bytes, _ = eng.memory_info()
    ds.free()
    t_load = time.perf_counter() - t_setup - t_gen
    log(f"[rank {rank}] shard {args.rows} x {D}, nnz/row {args.nnz}: generated {t_gen:.1f}s, resident "
        f"{train_bytes / 2**30:.2f} GiB in {t_load:.1f}s, {nb} batches/epoch")

    def run(k0, k):
        for i in range(k0, k0 + k):
            eng.train_step(i % nb, args.lr, 1.0, dlr.MODE_SYNC_MEAN)

    run(0, args.warmup)
    eng.sync()

    def barrier():
        if distributed:
            dist.barrier()

    def timed(k0, instrumented):
        """K steps bracketed by barrier + device sync on both sides; returns
        the max-over-ranks wall time."""
        eng.timing(instrumented)
        barrier()
        eng.sync()
        if torch is not None and torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(k0, args.steps)
        eng.sync()
        if torch is not None and torch.cuda.is_available():
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        barrier()
        if distributed:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # Pass 1 (the throughput): no per-kernel events in the launch stream.
    el = timed(args.warmup, False)
    # Pass 2: the same K steps with a HIP-event pair around every kernel on
    # the engine's stream -> per-kernel average durations for the roofline.
    el_instr = timed(args.warmup + args.steps, True)
    kt = {name: eng.kernel_time(i) for name, i in
          [("margin", dlr.TIMER_MARGIN), ("grad_update", dlr.TIMER_GRAD), ("merge", dlr.TIMER_UPDATE),
           ("exchange", dlr.TIMER_EXCHANGE), ("step", dlr.TIMER_STEP)]}
    eng.timing(False)
    samples = world * args.steps * B
    value = samples / el
    avg_us = {k: (ms / n * 1000.0 if n else 0.0) for k, (ms, n) in kt.items()}
    kern_us = avg_us["margin"] + avg_us["grad_update"] + avg_us["merge"]
    step_bytes = alg_bytes_per_step(B, args.nnz, D)
    achieved = step_bytes / (kern_us * 1e-6) / 1e9 if kern_us > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("workload_key") == f"D{D}_nnz{args.nnz}_B{B}":
                traffic = tj.get("hbm_bytes_per_step")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, D)
        except Exception as e:  # the baseline is a report, never the product
            log(f"cpu baseline failed: {e}")
    eng.close()

    if rank == 0:
        line = {
            "metric": "training samples/sec (whole node)",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1000.0, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded gen_data.py-shaped sparse rows, 4-decimal values; resident in HBM)",
            "config": {"workload": f"C2 sparse LR: {args.rows} rows/GPU x {D} features, {args.nnz} nnz/row, "
                                   f"batch {B}, sync SGD lr {args.lr}, C=1",
                       "rows_per_gpu": args.rows, "num_feature_dim": D, "nnz_per_row": args.nnz,
                       "batch_size": B, "parallelism": f"dp{world}"},
            "roofline": {
                "bound": "hbm",
                "kernel": "train step = k_margin_residual + k_grad (+ k_merge_update when N>1)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "alg_bytes_per_step": step_bytes,
                "kernel_avg_us": {k: round(v, 3) for k, v in avg_us.items()},
                "timing": "kernel averages from a second pass of the same K steps with HIP events on the "
                          "engine stream; value from the first, un-instrumented pass",
                "instrumented_ms_per_step": round(el_instr / args.steps * 1000.0, 5),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
