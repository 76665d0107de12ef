#!/usr/bin/env python
"""Where the C2 step's time goes over a bench process's life (VERDICT r4
weak #5): consecutive bracketed passes of the bench's step (sync on both
sides), each pass's ms/step, with the sweep launches' dispatch-stamped
durations and start-to-start intervals for every pass (smcdet_launch_timing).
A kernel that speeds up from pass to pass is the chip's clock (DVFS); gaps
that shrink are the host.  Variants: --gc-freeze (gc.freeze + disable before
the passes), --prewarm S (S seconds of back-to-back steps first).
    python scripts/warmup_probe.py [--passes 12] [--steps 20] [--gc-freeze] [--prewarm 0]
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smcdet_amd import _hip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--passes", type=int, default=12)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--gc-freeze", action="store_true")
ap.add_argument("--prewarm", type=float, default=0.0)
ap.add_argument("--events", action="store_true", help="dispatch-stamp every pass")
ap.add_argument("--host-times", action="store_true",
                help="per-step host enqueue times and GC collections of every pass")
a = ap.parse_args()

sys.argv = [sys.argv[0]]
bargs = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
s, mh, steps_per_step, _, cfg = bench.build_sampler(bargs, dev, 0)
s.initialize()
s._temper_reweight(with_resample=True)


def step():
    idx, s._pending_idx = s._pending_idx, None
    s._step(idx)


for _ in range(a.warmup):
    step()
torch.cuda.synchronize()
if a.prewarm > 0:
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.prewarm:
        for _ in range(20):
            step()
        torch.cuda.synchronize()
if a.gc_freeze:
    gc.collect()
    gc.freeze()
    gc.disable()
gc_events = []
if a.host_times:
    def _gc_cb(phase, info):
        gc_events.append((phase, info.get("generation"), time.perf_counter()))
    gc.callbacks.append(_gc_cb)
out = []
for p in range(a.passes):
    if a.events:
        _hip.launch_timing(a.steps)
    torch.cuda.synchronize()
    gc_events.clear()
    t0 = time.perf_counter()
    hs = []
    for _ in range(a.steps):
        h0 = time.perf_counter()
        step()
        hs.append(time.perf_counter() - h0)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps * 1e3
    row = {"pass": p, "ms_per_step": round(dt, 4)}
    if a.host_times:
        hs = np.array(hs) * 1e6
        row["host_us_p50"] = round(float(np.median(hs)), 1)
        row["host_us_max"] = round(float(hs.max()), 1)
        row["host_enqueue_ms_total"] = round(t_enq * 1e3, 3)
        gcs = [e for e in gc_events if e[0] == "start"]
        row["gc_collections"] = [g for _, g, _ in gcs]
        row["gc_us"] = [round((b[2] - a_[2]) * 1e6, 1) for a_, b in zip(gc_events[0::2], gc_events[1::2])]
    if a.events:
        ev = _hip.launch_timing_read(a.steps)
        st = _hip.launch_timing_starts(a.steps)
        _hip.launch_timing(0)
        row["kernel_ms_p50"] = round(float(np.median(ev)), 4)
        row["interval_ms_p50"] = round(float(np.median(np.diff(st))), 4) if len(st) > 1 else None
        row["interval_ms_max"] = round(float(np.max(np.diff(st))), 4) if len(st) > 1 else None
    out.append(row)
    print(json.dumps(row), flush=True)
print(json.dumps({"summary": {"first": out[0]["ms_per_step"], "last": out[-1]["ms_per_step"],
                              "min": min(r["ms_per_step"] for r in out),
                              "gc_freeze": a.gc_freeze, "prewarm_s": a.prewarm}}))
