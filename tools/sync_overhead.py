#!/usr/bin/env python3
"""Fixed cost of bench.py's timed region on one GPU: the two syncs that
close it, and K C2 steps for small K (the driver times K = 20).  A
development probe; prints microseconds."""
import os
import sys
import time

import torch  # noqa: F401  (the library binds to torch's HIP runtime)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dist-lr_amd"))
import distlr_amd as dlr  # noqa: E402

D, B = 1_000_000, 65536
ds = dlr.Dataset.generate(20 * B, D, 50, value_mode=1, seed=10, stream=1)
eng = dlr.Engine(D)
eng.set_weights(dlr.init_weight(D))
nb = eng.load_train(ds, B)
for i in range(50):
    eng.train_step(i % nb, 0.2, 1.0)
eng.sync()
torch.cuda.synchronize()


def region(k, both=True):
    eng.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        eng.train_step(i % nb, 0.2, 1.0)
    if both:
        eng.sync()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


for k in (0, 1, 2, 5, 20, 100):
    r = sorted(region(k) for _ in range(20))
    r1 = sorted(region(k, False) for _ in range(20))
    print(f"K={k:4d}: region median {r[10]:8.1f} us (engine + torch sync), {r1[10]:8.1f} us (torch sync only); "
          f"per step {((r[10] - sorted(region(0) for _ in range(5))[2]) / k if k else 0):.2f} us")
# after the GPU idled (as bench.py's timed pass does after loading the
# shard): 2 s of host sleep, W = 5 warmup steps, then K = 20 timed steps
for rep in range(3):
    time.sleep(2.0)
    for i in range(5):
        eng.train_step(i % nb, 0.2, 1.0)
    eng.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(5, 25):
        eng.train_step(i % nb, 0.2, 1.0)
    eng.sync()
    torch.cuda.synchronize()
    print(f"after 2 s idle + 5 warmup steps: K=20 region {(time.perf_counter() - t0) * 1e6:.1f} us")
t0 = time.perf_counter()
for i in range(1000):
    eng.train_step(i % nb, 0.2, 1.0)
t_host = (time.perf_counter() - t0) * 1e6 / 1000
eng.sync()
print(f"host issue rate: {t_host:.2f} us per train_step call (asynchronous)")
eng.close()
