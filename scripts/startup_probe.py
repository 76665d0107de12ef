#!/usr/bin/env python
"""Fixed cost of a timed region (C2): bench.py times K steps between two
synchronisations, so ms_per_step = GPU step + C/K.  For K = 20 steps:
the wall time, the GPU time per back-to-back step (events after step 1 and
after step K), the delay before step 1's kernels start (host enqueue after an
idle GPU), and the rest (the host noticing completion) -- with
torch.cuda.synchronize() alone and after spinning on an event query."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from smcdet_amd.sampler import SMCsampler  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    H, S, Np, K = 32, 10, 4096, 100
    model, prior, truth = bench.make_models(H, S)
    from smcdet_amd.kernel import SingleComponentMH as MH
    image = bench.synthetic_image(model, truth, H, 1, 1000, dev, max_sources=S)
    mh = MH(K, 0.1, 2.5, bench.M71["flux_lower"], bench.M71["flux_upper"])
    s = SMCsampler(image, H, prior, model, mh, Np, 0.5, "systematic",
                   bench.M71["flux_detection_threshold"], 10 ** 9, print_every=10 ** 9,
                   seed=12345, device=dev)
    s.initialize()
    s._temper_reweight(with_resample=True)

    def step():
        idx, s._pending_idx = s._pending_idx, None
        s._step(idx)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    out = {"rows": []}
    main_stream = torch.cuda.current_stream(dev)

    def spin():
        ev = torch.cuda.Event()
        ev.record(main_stream)
        while not ev.query():
            pass

    for rep in range(4):
        for mode in ("sync", "spin"):
            k = 20
            torch.cuda.synchronize()
            e0, e0b, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            t0 = time.perf_counter()
            e0.record(main_stream)
            step()
            e0b.record(main_stream)
            t1 = time.perf_counter()
            for _ in range(k - 1):
                step()
            e1.record(main_stream)
            if mode == "spin":
                spin()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            gpu = e0.elapsed_time(e1)
            g = e0b.elapsed_time(e1) / (k - 1)  # back-to-back steps: GPU time per step
            row = dict(mode=mode, k=k, wall_ms=(t2 - t0) * 1e3, event_ms=gpu, gpu_step_ms=g,
                       wall_minus_k_steps_us=((t2 - t0) * 1e3 - k * g) * 1e3,
                       first_step_start_delay_us=(e0.elapsed_time(e0b) - g) * 1e3,
                       wall_minus_event_us=((t2 - t0) * 1e3 - gpu) * 1e3,
                       first_enqueue_us=(t1 - t0) * 1e6)
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    a = time.perf_counter()
    torch.cuda.synchronize()
    out["idle_sync_us"] = (time.perf_counter() - a) * 1e6
    print(json.dumps(out))


if __name__ == "__main__":
    main()
