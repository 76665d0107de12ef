#!/usr/bin/env python
"""cProfile of the bench's C2 step on the host (enqueue cost per SMC step):
200 steps after warm-up, the top functions by own time."""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

sys.argv = [sys.argv[0]]
a = bench.parse()
dev = torch.device("cuda", 0)
s, mh, _, _, _ = bench.build_sampler(a, dev, 0)
s.initialize()
s._temper_reweight(with_resample=True)


def step():
    idx, s._pending_idx = s._pending_idx, None
    s._step(idx)


for _ in range(20):
    step()
torch.cuda.synchronize()
# host enqueue time per step (GPU far behind: the queue never drains here)
t = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    t.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
print("first step after a sync (host us):", [round(x * 1e6, 1) for x in t])
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(200):
    step()
pr.disable()
el = time.perf_counter() - t0
torch.cuda.synchronize()
print(f"host time per step under cProfile: {el / 200 * 1e6:.1f} us")
out = io.StringIO()
pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(25)
print(out.getvalue())
