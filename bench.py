#!/usr/bin/env python3
"""bench.py -- whole-node training throughput of the dist-lr hot path.

Workload (BASELINE.json configs[1], "C2"): synthetic sparse LR, 10M samples
x 1M features, 50 distinct uniform columns per row, 4-decimal values in
(0,1] (gen_data.py-shaped, seeded), batch 65,536 rows, sync SGD lr 0.2,
C = 1.  One step = one LR::Train batch: margin + sigmoid + residual, Xᵀr
gradient + L2, (exchange), SGD update.  Weak scaling: every rank trains its
own 10M-row shard (rank r = part-00{r+1}, like main.cc:158).

  python bench.py [--gpus N --steps K --warmup W] [--config c1|c2|c3|c4|c4s|c5]

N > 1: one process per GPU (rank r on GPU r, its own shard), RCCL over
xGMI for the exchange.  Launched either by torch.distributed.run (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* in the environment) or, without those,
by this script itself: the parent starts N rank processes with that
environment and never touches the GPU (or imports torch); `--spawn` takes
the same launcher path at N = 1.

Prints ONE JSON line on rank 0 (stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dist-lr_amd"))

torch = dist = dlr = np = None  # imported in the rank processes only (see main)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs measured here.  c2 is the default
# (configs[1], the headline single-GPU workload); the others are run with
# --config for their own bench lines.
CONFIGS = {
    # C1: examples/local.sh's a9a-shaped worker shard (D = 123, 14 binary
    # features/row, 8,140 rows per part file, B = -1: one full-shard step per
    # epoch); latency-bound, reported in absolute terms
    "c1": dict(rows=8140, features=123, nnz=14, batch=-1, value_mode=0, steps=2000, warmup=50,
               label="C1 local.sh a9a-shaped LR"),
    "c2": dict(rows=10_000_000, features=1_000_000, nnz=50, batch=65536, value_mode=1, steps=1000, warmup=50,
               label="C2 sparse LR"),
    # C3: per-GPU shard of the 100M-row Criteo-shaped set (8 GPUs); one step
    # = the full shard (B = -1, local.sh's batching), hashed Zipf fields
    "c3": dict(rows=12_500_000, features=1 << 24, nnz=39, batch=-1, value_mode=0, steps=10, warmup=2,
               label="C3 Criteo-shaped hashed LR", kind="hashed"),
    # C4: dense 4,096 fp32 features; 20M rows over 8 GPUs = 2.5M rows/GPU
    # (41 GB resident; a single GPU cannot hold all 20M rows: 328 GB)
    "c4": dict(rows=2_500_000, features=4096, nnz=4096, batch=65536, value_mode=1, steps=100, warmup=5,
               label="C4 dense LR", kind="dense"),
    "c5": dict(rows=1_024_000, features=1 << 28, nnz=10, batch=1024, value_mode=0, steps=200, warmup=10,
               label="C5 high-dim ultra-sparse LR"),
    # C4 on ONE GPU as SURVEY 8(d) states it: the rows do not fit in HBM, so
    # they stay in pinned host memory and each batch is staged over PCIe
    # (streamed residency); a 2.5M-row host shard stands in for the 20M rows
    # (the rate is per batch and does not depend on the shard's length)
    "c4s": dict(rows=2_500_000, features=4096, nnz=4096, batch=65536, value_mode=1, steps=40, warmup=4,
                label="C4 dense LR, streamed from host", kind="dense", residency="stream"),
    # C2 with the sparse shard kept in page-locked host memory and every
    # batch's CSR + column-major slices staged over PCIe (K1 streaming: what
    # a shard larger than HBM runs as; forced here on a shard that fits)
    "c2s": dict(rows=10_000_000, features=1_000_000, nnz=50, batch=65536, value_mode=1, steps=200, warmup=10,
                label="C2 sparse LR, streamed from host", residency="stream"),
}
# C1 end to end: bin/distlr running examples/local.sh's
# job (W = 2 workers, 100 epochs, B = -1, Test every 10; local.sh:12-19,
# main.cc:157-169) as a child process, timed beside the reference-structure
# CPU run of the same job on the same files -- handled by run_c1_e2e, before
# this process touches the GPU.
CONFIGS["c1e2e"] = dict(rows=8140, features=123, nnz=14, batch=-1, value_mode=0, steps=100, warmup=1,
                        label="C1 local.sh job end to end (bin/distlr)", kind="e2e")
# Every config runs in the engine's default, REFERENCE summation order
# (dlr_set_summation_order: every margin one chain in column order, every
# gradient column one chain in batch-row order, lr.cc:35-40/108-112 --
# bitwise the oracle).  c3f / c4f: the same workloads in the opt-in FAST
# order (deterministic reordered sums for the ~10^5-10^6-add chains,
# DESIGN.md 3), for the price of the reference order.
CONFIGS["c3f"] = dict(CONFIGS["c3"], label="C3 Criteo-shaped hashed LR, FAST summation order", order="fast")
CONFIGS["c4f"] = dict(CONFIGS["c4"], label="C4 dense LR, FAST summation order (fused blocked pass)", order="fast")
PCIE_PEAK_GBS = 63.0  # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s (spec)


def make_shard(args, n_rows: int, stream: int):
    if args.kind == "dense":
        return dlr.DenseDataset.generate(n_rows, args.features, seed=10, stream=stream)
    if args.kind == "hashed":
        return dlr.Dataset.generate_hashed(n_rows, args.features, args.nnz, seed=10, stream=stream)
    return dlr.Dataset.generate(n_rows, args.features, args.nnz, value_mode=args.value_mode, seed=10, stream=stream)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="BASELINE config (c1e2e: local.sh's job end to end through bin/distlr)")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--rows", type=int, default=None, help="training rows per GPU shard")
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--value-mode", type=int, default=None,
                    help="override the config's values (0: unit, 1: 4-decimal fp32; Dataset.generate)")
    ap.add_argument("--lr", type=float, default=0.2)
    ap.add_argument("--xpieces", type=int, default=0,
                    help="N > 1: pieces of the overlapped all-gather (dlr_set_exchange_pieces; 0 = auto, "
                         "one per 4 MiB of a rank's key range, 1 to 4)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-pass", action="store_true",
                    help="skip the per-stage roofline pass (PMC runs: every kernel then belongs to a whole step; "
                         "the roofline uses the step time)")
    ap.add_argument("--mode", choices=["mean", "last", "async"], default="mean",
                    help="server update rule (main.cc:57-84): sync mean (default), sync last push, async")
    ap.add_argument("--spawn", action="store_true", help="use the process launcher even at --gpus 1")
    ap.add_argument("--loopback-ranks", type=int, default=0,
                    help="W > 1: an N > 1 exchange cost estimate on ONE GPU -- W ranks of the loopback "
                         "transport (dlr_create_group, one thread each) run the world-W step; prints the "
                         "exchange/merge microseconds per step with and without the overlap (not a "
                         "throughput line)")
    ap.add_argument("--launcher-check", action="store_true",
                    help="ranks rendezvous over gloo and rank 0 prints the ranks it saw, no GPU work (CPU tests)")
    ap.add_argument("--dump-weights", default=None,
                    help="write each rank's weights after the timed passes to PATH.rank<r> (tests)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per step (written by tools/pmc_traffic.py; default "
                         "profiles/traffic.json for c2, profiles/traffic_<config>.json otherwise)")
    args = ap.parse_args()
    if args.traffic_json is None:
        args.traffic_json = os.path.join(ROOT, "profiles", "traffic.json" if args.config == "c2"
                                         else f"traffic_{args.config}.json")
    cfg = CONFIGS[args.config]
    for k in ("rows", "features", "nnz", "batch", "steps", "warmup"):
        if getattr(args, k) is None:
            setattr(args, k, cfg[k])
    if args.value_mode is None:
        args.value_mode = cfg["value_mode"]
    args.label = cfg["label"]
    args.kind = cfg.get("kind", "uniform")
    args.residency = cfg.get("residency", "auto")
    args.env = cfg.get("env", {})
    args.order = cfg.get("order", "reference")
    return args


def alg_bytes_per_step(B: int, nnz: float, D: int, dense: bool = False, unit: bool = False) -> int:
    """sparse 8*nnz + 8 bytes per sample (int32 col + fp32
    val per nnz; row offset + label per row), dense 4*D + 4 (the row + its
    label), + 8*D/B per sample (dense-L2 weight read + write), times the B
    samples of one step.  A unit-valued shard (every value 1.0f: C3, C5)
    has no values to read: 4*nnz + 8."""
    per = 4 * D + 4 if dense else (4 if unit else 8) * nnz + 8
    return int(round(B * per + 8 * D))


def cpu_baseline(args, D: int) -> dict:
    """the reference's CPU path with its own cost structure
    (oracle/ref_loop.cc: local.sh's worker threads + in-process server,
    per-epoch re-parse into dense samples, lr.cc:35-39's O(B*D^2) loop with
    by-value copies; its weights are bitwise the oracle's).  Calibrated in
    the build container against the verbatim reference (BASELINE.md 2:
    52.9k samples/s at W = 1; this restatement 52.3k).
    c1: local.sh's job itself (W = 2 threads, B = -1, test every 10 epochs)
    for a bounded number of epochs.  Other configs cannot run it (a dense
    sample is D floats, a step O(B*D^2)): the lr.cc:35-39 loop body is
    timed at the config's D and the per-sample cost (D of them) reported."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_baselines as cb  # baseline only, never the product
    if args.config == "c1":
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            for sub in ("train", "test", "models"):
                os.makedirs(os.path.join(d, sub))
            for p in range(2):
                make_shard(args, args.rows, p + 1).write_libsvm(os.path.join(d, "train", f"part-00{p + 1}"))
            make_shard(args, 16281, 100).write_libsvm(os.path.join(d, "test", "part-001"))
            epochs = 60
            _, steps, sec, _, _ = cb.reference_local_run(d, 2, D, epochs, -1, 10, args.lr, 0)
        return {"value": round(steps / sec, 1), "unit": "samples/s", "cores": 2, "host_cpus": os.cpu_count(),
                "kind": "port",
                "sample": f"local.sh topology (2 worker threads + in-process server, examples/local.sh:12-19): "
                          f"{epochs} epochs of 2 x {args.rows} rows, B = -1, per-epoch re-parse, test every 10 "
                          f"epochs on 16,281 rows; {steps} sample-steps in {sec:.1f} s (oracle/ref_loop.cc: "
                          f"lr.cc/main.cc loop structure, weights bitwise the oracle's)"}
    iters = 8
    while True:
        t = cb.reference_inner_cost(D, 4, iters)
        if t * iters >= 2.0 or iters >= 1 << 30:
            break
        iters *= 4
    per_sample = t * D  # lr.cc:35-39 runs the body D times per sample (one per column j)
    return {"value": float(f"{1.0 / per_sample:.4g}"), "unit": "samples/s", "cores": 1, "host_cpus": os.cpu_count(),
            "kind": "port",
            "sample": f"extrapolated: {iters} iterations of lr.cc:35-39's loop body at D = {D} (two by-value "
                      f"copies of a {D}-float sample + the O(D) margin) took {t * 1e6:.3g} us each; a "
                      f"sample-step is D = {D} of them ({per_sample:.3g} s); one worker thread "
                      f"(oracle/ref_loop.cc; the reference cannot hold this config: dense samples)"}


def cpu_baseline_build(args, D: int) -> dict:
    """BASELINE.md 3.2 -- "build CPU path, not reference": an efficient
    OpenMP trainer (oracle/lr_cpu_omp.c) on the host's CPU share
    (OMP_NUM_THREADS), over a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_baselines as cb  # baseline only, never the product
    B = args.batch if args.batch > 0 else min(args.rows, 200_000)  # full-shard configs: B = -1 over <= 200k rows
    n_rows = 4 * B if args.batch > 0 else B
    ds = make_shard(args, n_rows, 1)
    w = dlr.init_weight(D)
    done, el = 0, 0.0
    if args.kind == "dense":
        X, lab = ds.arrays()
        step = lambda k: cb.omp_train_dense(X, lab, B, w, args.lr, 1.0, k, 1)  # noqa: E731
    else:
        rp, col, val, lab = ds.csr()
        unit = bool(np.all(val == 1.0))
        step = lambda k: cb.omp_train_csr(rp, col, None if unit else val, lab, D, B, w, args.lr, 1.0, k, 1)  # noqa: E731
    step(0)  # first touch of the working set
    while el < args.cpu_seconds and done < 100_000:
        el += step(done)
        done += 1
    return {"value": round(done * B / el, 1), "unit": "samples/s", "cores": cb.omp_threads(),
            "host_cpus": os.cpu_count(), "kind": "build CPU path, not reference",
            "sample": f"{done} steps of B = {B} over {n_rows} rows (D = {D}, {args.nnz} nnz/row) in {el:.1f} s, "
                      f"OpenMP {cb.omp_threads()} threads (oracle/lr_cpu_omp.c)"}


def run_c1_e2e(args) -> None:
    """local.sh's job through the drop-in driver: `bin/distlr` with local.sh's
    environment and 2 workers (two loopback ranks on GPU 0), args.steps
    epochs, timed from process start to exit (parse, GPU init, training,
    tests, model files) and over its epoch loops (DISTLR_TIMING), `warmup`
    runs first; then the reference-structure CPU run of the same job on the
    same files (oracle/ref_loop.cc, 2 worker threads).  value = training
    samples (2 x rows x epochs) / end-to-end seconds."""
    global dlr
    import re
    import tempfile
    import distlr_amd as dlr  # noqa: F811  -- host-only entry points here (generator, model text): no GPU
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_baselines as cb  # baseline only, never the product
    W, D, epochs = 2, args.features, args.steps
    exe = os.path.join(ROOT, "dist-lr_amd", "bin", "distlr")
    with tempfile.TemporaryDirectory() as d:
        for sub_ in ("train", "test", "models"):
            os.makedirs(os.path.join(d, sub_))
        for p in range(W):
            make_shard(args, args.rows, p + 1).write_libsvm(os.path.join(d, "train", f"part-00{p + 1}"))
        make_shard(args, 16281, 100).write_libsvm(os.path.join(d, "test", "part-001"))
        env = dict(os.environ, DATA_DIR=d, NUM_FEATURE_DIM=str(D), NUM_ITERATION=str(epochs), BATCH_SIZE="-1",
                   TEST_INTERVAL="10", SYNC_MODE="1", LEARNING_RATE=str(args.lr), DMLC_NUM_WORKER=str(W),
                   DISTLR_TIMING="1")
        env.pop("DMLC_ROLE", None)
        runs = []
        for _ in range(args.warmup + 1):
            t0 = time.perf_counter()
            r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=600)
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                sys.exit(f"bin/distlr failed ({r.returncode}): {r.stderr[-2000:]}")
            loops = [float(x) for x in re.findall(r"epoch loop ([0-9.eE+-]+) s", r.stderr)]
            acc = re.findall(r"Iteration (\d+), accuracy: (\S+)", r.stdout)
            runs.append((wall, max(loops) if loops else None, acc))
        with open(os.path.join(d, "models", "part-001")) as f:
            model0 = f.read()
        w_ref, steps, sec, corr, n_test = cb.reference_local_run(d, W, D, epochs, -1, 10, args.lr, 0)
    wall, loop, acc = runs[-1]
    samples = W * args.rows * epochs
    ref_acc = f"{cb_accuracy(corr, n_test)}"
    line = {
        "metric": "training samples/sec (whole node)",
        "value": round(samples / wall, 1),
        "unit": "samples/s",
        "n_gpus": 1,
        "steps": epochs,
        "warmup": args.warmup,
        "ms_per_step": round(wall / epochs * 1000.0, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded gen_data.py-shaped a9a-like libsvm text files, binary values)",
        "config": {"workload": f"{args.label}: examples/local.sh's job -- {W} workers x {args.rows} rows x {D} "
                               f"features, {args.nnz} nnz/row, B = -1, {epochs} epochs, Test every 10 epochs on "
                               f"16,281 rows, SYNC_MODE=1, LEARNING_RATE={args.lr}",
                   "name": "c1e2e", "driver": "dist-lr_amd/bin/distlr (main.cc's drop-in), loopback group of 2 "
                                              "ranks on GPU 0", "parallelism": "dp2 (one GPU)"},
        "end_to_end_s": round(wall, 4),
        "epoch_loop_s": loop,
        "epoch_loop_samples_per_s": round(samples / loop, 1) if loop else None,
        "first_run_s": round(runs[0][0], 4),
        "step": "one epoch of local.sh's job = one B = -1 step per worker (+ a Test every 10 epochs)",
        "accuracy_lines": [f"Iteration {i}, accuracy: {a}" for i, a in acc],
        "reference_final_accuracy": ref_acc,
        "final_accuracy_equal": bool(acc) and acc[-1][1] == ref_acc,
        "model_part001_equals_reference_weights": model0 == dlr.format_model(w_ref),
        "roofline": None,
        "roofline_note": "latency-bound job (one 8,140-row step per worker per epoch): no HBM roofline; the "
                         "kernels' own line is --config c1",
        "cpu_baseline": {"value": round(steps / sec, 1), "unit": "samples/s", "cores": W, "host_cpus": os.cpu_count(),
                         "kind": "port",
                         "sample": f"the same job on the same files: {W} worker threads + in-process server, "
                                   f"per-epoch re-parse, lr.cc/main.cc loop structure (oracle/ref_loop.cc), "
                                   f"{epochs} epochs, {steps} sample-steps in {sec:.2f} s"},
    }
    print(json.dumps(line), flush=True)


def cb_accuracy(correct: int, n: int) -> str:
    """lr.cc:59-62's accuracy text (ostream %g of the float ratio)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the checker's formatter
    return oracle.format_g(oracle.accuracy(correct, n))


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch(n: int) -> int:
    """Starts n rank processes of this script (rank r -> GPU r), each with
    the torch.distributed.run environment, and waits for them.  The parent
    never imports torch or the engine: it only forks + execs fresh
    interpreters, before anything has touched a GPU.  Rank 0 writes the JSON
    line to the inherited stdout.  If a rank fails, the others are stopped."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLR_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log(f"bench launcher: rank {procs.index(p)} exited with {code}; stopping the others")
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    args = parse_args()
    if args.loopback_ranks > 1:
        if args.gpus != 1 or "WORLD_SIZE" in os.environ:
            sys.exit("--loopback-ranks runs W ranks on one GPU: --gpus 1, no launcher")
        run_loopback(args)
        return
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.spawn):
        sys.exit(launch(args.gpus))
    run_rank(args)


def run_loopback(args):
    """The world-W step on ONE GPU through the loopback transport (DESIGN.md
    8): W contexts on device 0, one host thread each, the exchange's
    collectives as device-to-device copies ordered by events.  What it
    measures: the exchange's own work per step -- the key-range all-to-all
    and all-gather as HBM copies (W - 1 peer blocks each way), the
    rank-ordered merge, the next batch's pass 1 regrouped around the pieces
    -- and how much of it the overlap hides.  What it cannot measure: xGMI
    and RCCL latency (no multi-GPU box in this pool).  The W ranks share the
    GPU, so ms_per_step is W ranks' compute."""
    global dlr, np
    import threading
    import numpy as np  # noqa: F811
    try:
        import torch  # noqa: F401  -- the library binds to torch's HIP runtime
    except Exception:  # pragma: no cover
        pass
    import distlr_amd as dlr  # noqa: F811
    W, D, B = args.loopback_ranks, args.features, args.batch
    t0 = time.perf_counter()
    shards = []
    for r in range(W):  # (a line per shard: a long generation is not a hang)
        shards.append(make_shard(args, args.rows, r + 1))
        log(f"loopback: shard {r + 1} of {W} generated ({time.perf_counter() - t0:.1f}s)")
    log(f"loopback: {W} shards of {args.rows} x {D} generated in {time.perf_counter() - t0:.1f}s")
    engines = dlr.Engine.create_group(D, W, 0)
    w0 = dlr.init_weight(D)
    res = [None] * W
    errors = [None] * W
    bar = threading.Barrier(W)

    def rank_main(r):
        eng = engines[r]
        try:
            eng.set_exchange_pieces(args.xpieces)
            eng.set_weights(w0)
            nb = eng.load_train_dense(shards[r], B) if args.kind == "dense" else eng.load_train(shards[r], B)
            shards[r].free()
            log(f"loopback: rank {r} loaded ({time.perf_counter() - t0:.1f}s)")
            k = 0

            def steps(n, instrumented):
                nonlocal k
                eng.timing(instrumented)
                bar.wait()
                eng.sync()
                bar.wait()
                ta = time.perf_counter()
                for _ in range(n):
                    eng.train_step(k % nb, args.lr, 1.0, dlr.MODE_SYNC_MEAN)
                    k += 1
                eng.sync()
                el = time.perf_counter() - ta
                out = {name: eng.kernel_time(i) for name, i in
                       [("exchange", dlr.TIMER_EXCHANGE), ("merge", dlr.TIMER_UPDATE), ("margin", dlr.TIMER_MARGIN),
                        ("grad_update", dlr.TIMER_GRAD)]} if instrumented else {}
                bar.wait()
                return el, out

            def per_step(t):
                ms, n = t
                return round(ms / max(1, n) * 1000.0, 3)

            steps(args.warmup, False)
            el_on, _ = steps(args.steps, False)
            _, kt_on = steps(args.steps, True)
            overlap, pieces = eng.exchange_overlap(), eng.exchange_pieces()
            off = None
            if overlap:
                eng.set_exchange_overlap(False)  # collective: every rank calls it here
                el_off, _ = steps(args.steps, False)
                _, kt_off = steps(args.steps, True)
                eng.set_exchange_overlap(True)
                off = {"ms_per_step": round(el_off / args.steps * 1000.0, 5),
                       "exchange_us_per_step": per_step(kt_off["exchange"]),
                       "margin_us_per_step": per_step(kt_off["margin"])}
            cnt = eng.stage_counters()  # (since the load: every step above)
            res[r] = {"counters": cnt, "steps_run": k,
                      "ms_per_step": round(el_on / args.steps * 1000.0, 5), "overlap": bool(overlap),
                      "pieces": pieces, "exchange_us_per_step": per_step(kt_on["exchange"]),
                      "merge_us_per_step": per_step(kt_on["merge"]), "margin_us_per_step": per_step(kt_on["margin"]),
                      "gradient_us_per_step": per_step(kt_on["grad_update"]), "without_overlap": off,
                      "weights_sha1": hashlib.sha1(eng.get_weights().tobytes()).hexdigest()}
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors[r] = e
            eng.comm_abort(f"rank {r}: {e}")
            try:
                bar.abort()
            except Exception:
                pass

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in engines:
        e.close()
    for r, e in enumerate(errors):
        if e is not None:
            raise RuntimeError(f"loopback rank {r} failed") from e
    r0 = res[0]
    line = {
        "metric": "exchange cost estimate (loopback transport, W ranks on one GPU)",
        "ranks": W, "config": {"name": args.config, "rows_per_rank": args.rows, "num_feature_dim": D,
                               "nnz_per_row": args.nnz, "batch_size": B},
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step_all_ranks": r0["ms_per_step"],
        "exchange_us_per_step": r0["exchange_us_per_step"], "merge_us_per_step": r0["merge_us_per_step"],
        "margin_us_per_step": r0["margin_us_per_step"], "gradient_us_per_step": r0["gradient_us_per_step"],
        "overlap": r0["overlap"], "pieces": r0["pieces"], "without_overlap": r0["without_overlap"],
        "per_rank_exchange_us": [x["exchange_us_per_step"] for x in res],
        # the in-launch hand-offs under the world > 1 stream set (dlr_stage_counters, every rank, all steps
        # since the load): hot-chain give-ups must be 0
        "counters": {"steps_per_rank": r0["steps_run"],
                     "hot_chain_launches_per_step": round(r0["counters"]["hot_chain_launches"] / max(1, r0["steps_run"]), 3),
                     "hot_giveups_all_ranks": sum(x["counters"]["hot_giveups"] for x in res),
                     "cowait_serialised_all_ranks": sum(x["counters"]["cowait_serialised"] for x in res),
                     "mg_demoted_all_ranks": sum(x["counters"]["mg_demoted"] for x in res)},
        "ranks_agree": len({x["weights_sha1"] for x in res}) == 1,
        "note": "the W ranks share one GPU (their compute is serialised on it); the collectives are "
                "event-ordered device copies, so xGMI/RCCL latency is NOT in these numbers: the exchange's "
                "own work (copies, rank-ordered merge, pass-1 regrouping) and what the overlap hides",
    }
    print(json.dumps(line), flush=True)


def run_rank(args):
    global torch, dist, dlr, np
    import numpy as np  # noqa: F811
    try:
        import torch  # noqa: F811  -- loaded first: the library binds to torch's HIP runtime
        import torch.distributed as dist  # noqa: F811
    except Exception:  # pragma: no cover
        torch = dist = None
    import distlr_amd as dlr  # noqa: F811

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.kind == "e2e":
        if world != 1:
            sys.exit("--config c1e2e runs bin/distlr's own 2-worker job: --gpus 1")
        run_c1_e2e(args)  # before anything here touches the GPU (the child owns it)
        return
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    distributed = world > 1
    if torch is not None and not args.launcher_check and torch.cuda.is_available():
        torch.cuda.set_device(local)  # torch.cuda.synchronize() below then waits on this rank's GPU only
    if distributed:
        dist.init_process_group("gloo")   # control plane only; data path is RCCL inside the library
    if args.launcher_check:
        seen = [None] * world
        if distributed:
            dist.all_gather_object(seen, {"rank": rank, "local_rank": local, "pid": os.getpid()})
        else:
            seen = [{"rank": rank, "local_rank": local, "pid": os.getpid()}]
        if rank == 0:
            print(json.dumps({"launcher_check": seen, "world": world}), flush=True)
        if distributed:
            dist.destroy_process_group()
        return
    os.environ.update(args.env)
    D, B = args.features, args.batch
    mode = {"mean": dlr.MODE_SYNC_MEAN, "last": dlr.MODE_SYNC_LAST, "async": dlr.MODE_ASYNC}[args.mode]

    uid = None
    if distributed:
        obj = [dlr.get_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]

    t_setup = time.perf_counter()
    ds = make_shard(args, args.rows, rank + 1)
    if args.kind == "dense":
        nnz_avg = float(D)
    else:
        nnz_avg = ds.info()[1] / max(1, args.rows)    # hashed rows lose a few duplicate fields
    t_gen = time.perf_counter() - t_setup
    eng = dlr.Engine(D, device=local, rank=rank, world=world, unique_id=uid)
    eng.set_summation_order(dlr.ORDER_FAST if args.order == "fast" else dlr.ORDER_REFERENCE)
    eng.set_exchange_pieces(args.xpieces)
    eng.set_weights(dlr.init_weight(D))
    if args.residency != "auto":
        eng.set_residency({"device": dlr.RESIDENCY_DEVICE, "stream": dlr.RESIDENCY_STREAM}[args.residency])
    nb = eng.load_train_dense(ds, B) if args.kind == "dense" else eng.load_train(ds, B)
    streamed = eng.train_residency() == dlr.RESIDENCY_STREAM
    train_bytes, _ = eng.memory_info()
    if not (streamed and args.kind == "dense"):
        ds.free()   # a streamed DENSE shard reads these host rows in place every step
    t_load = time.perf_counter() - t_setup - t_gen
    layout = "dense" if args.kind == "dense" else \
        {dlr.LAYOUT_CLASSIC: "classic", dlr.LAYOUT_LDS: "lds", dlr.LAYOUT_TOUCHED: "touched"}[eng.train_layout()]
    band_rows = eng.train_band_rows() if args.kind != "dense" else 0
    # which summation order the numbers below are for: what
    # the loaded shard's kernels actually use (dlr_summation_order)
    order_name = "reference" if eng.summation_order() == dlr.ORDER_REFERENCE else "fast"
    if eng.summation_order() == dlr.ORDER_REFERENCE:
        order = "reference: one chain per row (margin) and per column (gradient), lr.cc:35-40/108-112 -- bitwise"
    elif args.kind == "dense":
        order = ("FAST (opt-in): margins as 64 lane partials + butterfly, gradient per 256-row chunk + chunk "
                 "order (deterministic; DESIGN.md 3.3)")
    else:
        order = ("FAST (opt-in): reference except long columns (> 2,048 entries): 16,384-row phase pieces "
                 "combined by a fixed tree (deterministic; DESIGN.md 3.1)")
    row_rounds = eng.train_row_rounds() if args.kind != "dense" else 0
    margin_kind = "dense rows" if args.kind == "dense" else \
        ["gathers", "product margin (pass 1 separate)",
         "product margin (pass 1 fused into the previous step's gradient)",
         "product margin (pass 1 fused into the previous step's gradient, pass 2 into this step's)"][
            eng.train_product_margin()]
    log(f"[rank {rank}] shard {args.rows} x {D}, nnz/row {args.nnz}: generated {t_gen:.1f}s, "
        f"{'streamed from host' if streamed else 'resident'} {train_bytes / 2**30:.2f} GiB in {t_load:.1f}s, "
        f"{nb} batches/epoch, gradient layout {layout}")

    def run(k0, k):
        for i in range(k0, k0 + k):
            eng.train_step(i % nb, args.lr, 1.0, mode)

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

    # Pass 1: K steps with a HIP-event pair around every launch on the
    # engine's stream -> the step breakdown (exchange included, N>1).
    # Pass 2 (the throughput, `value`): the next K steps, no per-kernel
    # events in the launch stream.  The instrumented pass runs first so that
    # the throughput pass does not start on a GPU whose clocks are still
    # ramping from the idle host-side setup ("Short timed
    # regions"); both are K real steps bracketed the same way.
    el_instr = timed(args.warmup, True)
    kt = {name: eng.kernel_time(i) for name, i in
          [("margin", dlr.TIMER_MARGIN), ("grad_update", dlr.TIMER_GRAD), ("merge", dlr.TIMER_UPDATE),
           ("exchange", dlr.TIMER_EXCHANGE), ("step", dlr.TIMER_STEP)]}
    el = timed(args.warmup + args.steps, False)   # (timing(False) clears the event totals: read above)
    # Every rank holds the replicated weights after the same 2K (+W) steps:
    # their checksums must agree (and, with --dump-weights, the tests compare
    # them with the oracle's W-worker run).
    counters = eng.stage_counters()  # since the load: the warmup and both timed passes
    steps_run = args.warmup + 2 * args.steps
    w_fin = eng.get_weights()
    digest = hashlib.sha1(w_fin.tobytes()).hexdigest()
    if args.dump_weights:
        w_fin.tofile(f"{args.dump_weights}.rank{rank}")
    digests = [digest]
    if distributed:
        digests = [None] * world
        dist.all_gather_object(digests, digest)
    nranks, transport = eng.comm_info()
    # N > 1 with the product margin: the same K steps once more with the
    # exchange NOT overlapped with the next batch's pass 1 (plain all-gather,
    # pass 1 in the next margin), so the line shows what the overlap buys
    overlap = eng.exchange_overlap() if world > 1 else False
    xpieces = eng.exchange_pieces()
    no_overlap = None
    if overlap:
        eng.set_exchange_overlap(False)
        el_off = timed(args.warmup + 2 * args.steps, False)
        eng.timing(True)
        timed(args.warmup + 3 * args.steps, True)
        ex_off = eng.kernel_time(dlr.TIMER_EXCHANGE)
        mg_off = eng.kernel_time(dlr.TIMER_MARGIN)
        eng.timing(False)
        eng.set_exchange_overlap(True)
        no_overlap = {"ms_per_step": round(el_off / args.steps * 1000.0, 5),
                      "exchange_us_per_step": round(ex_off[0] / max(1, ex_off[1]) * 1000.0, 3),
                      "margin_us_per_step": round(mg_off[0] / max(1, mg_off[1]) * 1000.0, 3)}
    # Pass 3 (the roofline): each kernel stage over K consecutive batches
    # between ONE event pair (no per-launch event overhead, comparable with
    # rocprofv3's kernel durations).  Runs after the measured passes: the
    # stages run without their partners and change the weights.
    # (A streamed shard is bound by the batch copies instead: no stage pass.)
    k0 = args.warmup + (4 if overlap else 2) * args.steps
    stage_us = {}
    if not streamed and not args.no_stage_pass:
        stage_us = {"margin": eng.stage_time(dlr.STAGE_MARGIN, k0 % nb, args.steps, args.lr) * 1000.0,
                    "gradient": eng.stage_time(dlr.STAGE_GRADIENT, k0 % nb, args.steps, args.lr) * 1000.0}
    if layout == "touched" and not args.no_stage_pass:
        stage_us["update"] = eng.stage_time(dlr.STAGE_UPDATE, k0 % nb, args.steps, args.lr) * 1000.0
    B_eff = B if B > 0 else args.rows                 # B = -1: the full shard per step
    samples = world * args.steps * B_eff
    value = samples / el
    avg_us = {k: (ms / n * 1000.0 if n else 0.0) for k, (ms, n) in kt.items()}
    # the step's kernels: stage averages, plus the key-range merge (N>1).
    # Where the step runs its stages beside each other (band mode: each band's
    # gradient and the hot chains on their own streams beside the next
    # band's margin) the stages' isolated times add up to more than the step
    # itself; the roofline then uses the step's own time
    stage_sum_us = sum(stage_us.values()) + (avg_us["merge"] if world > 1 and layout != "touched" else 0.0)
    step_us = el / args.steps * 1e6
    kern_us = min(stage_sum_us, step_us) if stage_sum_us > 0 else step_us
    time_basis = ("step time (no stage pass)" if stage_sum_us <= 0 else
                  "step time (stages overlap)" if stage_sum_us > step_us else "sum of the stage averages")
    unit = args.kind != "dense" and eng.train_unit_values()
    step_bytes = alg_bytes_per_step(B_eff, nnz_avg, D, args.kind == "dense", unit)
    achieved = step_bytes / (kern_us * 1e-6) / 1e9 if kern_us > 0 else 0.0
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if (tj.get("workload_key") == f"D{D}_nnz{args.nnz}_B{B}" and tj.get("layout", layout) == layout
                    and tj.get("summation_order", order_name) == order_name):
                traffic = tj.get("hbm_bytes_per_step")
        except Exception:
            traffic = None

    roofline = {
        "bound": "hbm",
        "kernel": "train step = margin (K2) + gradient (K3, + fused update) + update/merge (K4: dense L2 "
                  "pass for the touched layout, key-range merge when N>1)",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_source": (f"stored figure, not measured in this run: {os.path.relpath(args.traffic_json, ROOT)} "
                           "(rocprofv3 --pmc passes of this workload, tools/pmc_pass.sh + tools/pmc_traffic.py)")
                          if traffic is not None else None,
        "alg_bytes_per_step": step_bytes,
        "kernel_avg_us": {k: round(v, 3) for k, v in stage_us.items()},
        "time_basis": time_basis,
        "time_us": round(kern_us, 3),
        "step_breakdown_us": {k: round(v, 3) for k, v in avg_us.items()},
        "timing": "value: K un-instrumented steps; kernel_avg_us: each kernel stage over K consecutive "
                  "batches between one HIP-event pair on the engine stream (achieved = alg bytes / their "
                  "sum); step_breakdown_us: a pass of K steps with an event pair around every launch "
                  "(includes the exchange when N>1; event overhead ~2 us per launch)",
        "instrumented_ms_per_step": round(el_instr / args.steps * 1000.0, 5),
    }
    if streamed:
        # bound by the host->device batch copies: the engine's own count of
        # the bytes one batch's copies move (dlr_stream_bytes: dense, the
        # batch's rows; sparse, the coalesced CSR + block bases -- the LDS
        # layout is built on the device and never crosses PCIe), epoch mean
        h2d = eng.stream_bytes()[0]
        pcie = h2d / (el / args.steps) / 1e9
        roofline.update({"bound": "pcie", "kernel": "per-batch host->device staging (copy stream) overlapped "
                                                      "with the margin/gradient kernels of the previous batch",
                         "achieved": round(pcie, 2), "peak": PCIE_PEAK_GBS, "frac": round(pcie / PCIE_PEAK_GBS, 4),
                         "h2d_bytes_per_step": h2d, "hbm_kernels_gbs": round(achieved, 1) if kern_us > 0 else None})
        roofline["timing"] = "value and achieved: K un-instrumented steps (copy-bound); step_breakdown_us: " \
                             "the event pass (the margin interval includes the wait for the batch copy)"

    cpu = cpu_build = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, D)
        except Exception as e:  # the baseline is a report, never the product
            log(f"cpu baseline failed: {e}")
        try:
            cpu_build = cpu_baseline_build(args, D)
        except Exception as e:
            log(f"cpu build baseline failed: {e}")
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
            "data": f"synthetic (seeded gen_data.py-shaped {'dense' if args.kind == 'dense' else 'sparse'} rows, "
                    f"{'4-decimal' if args.value_mode else 'binary'} values; "
                    f"{'pinned host memory, staged per batch' if streamed else 'resident in HBM'})",
            "config": {"workload": f"{args.label}: {args.rows} rows/GPU x {D} features, {args.nnz} nnz/row, "
                                   f"batch {B}, sync SGD lr {args.lr}, C=1",
                       "name": args.config, "gradient_layout": layout + (f"+bands({band_rows} rows)" if band_rows else "") +
                       (f" (row-round gradient k_grad_rt, {row_rounds} rounds)" if row_rounds else ""),
                       "values": "unit (all 1.0f, not stored)" if unit else "fp32",
                       "margin": margin_kind,
                       "summation_order": order,
                       "rows_per_gpu": args.rows, "num_feature_dim": D, "nnz_per_row": args.nnz,
                       "batch_size": B, "parallelism": f"dp{world}"},
            "roofline": roofline,
            "exchange": {
                "transport": {dlr.TRANSPORT_NONE: "none (1 rank)", dlr.TRANSPORT_RCCL: "rccl",
                              dlr.TRANSPORT_LOOPBACK: "loopback"}[transport],
                "rccl_nranks": nranks if transport == dlr.TRANSPORT_RCCL else 0,
                "launcher": os.environ.get("DLR_BENCH_LAUNCHER") or
                            ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else
                             ("external" if distributed else "single process")),
                "us_per_step": round(avg_us["exchange"], 3),
                "overlap": ("the all-gather in pieces, the next batch's pass 1 formed slice group by slice group "
                            "as its weights land (us_per_step includes that pass 1; the margin then runs pass 2 only)"
                            if overlap else None),
                "pieces": xpieces,
                "without_overlap": no_overlap,
                "merge_us_per_step": round(avg_us["merge"], 3) if world > 1 else 0.0,
                "protocol": ("touched-list all-gather + rank-ordered merge" if layout == "touched" else
                             "key-range all-to-all + rank-ordered merge + in-place all-gather") if world > 1 else
                            "none",
                "weights_sha1": digest,
                "ranks_agree": len(set(digests)) == 1,
            },
            # the in-launch hand-offs (dlr_stage_counters over the warmup + both timed passes): hot-chain
            # give-ups must be 0; cowait_serialised counts launches ordered behind another context's
            "counters": {"steps": steps_run,
                         "hot_chain_launches_per_step": round(counters["hot_chain_launches"] / steps_run, 3),
                         "hot_giveups": counters["hot_giveups"],
                         "cowait_serialised": counters["cowait_serialised"],
                         "mg_demoted": counters["mg_demoted"]},
            "cpu_baseline": cpu,
            "cpu_baseline_build": cpu_build,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
