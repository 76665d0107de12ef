#!/usr/bin/env python
"""Host-side cost of one fused SMC step (C2): Python + ctypes time spent
issuing the MH sweep and the tile launch, against the GPU time of the step.
If the host issue time approaches the GPU time, the GPU idles between
kernels (the launch gaps seen in the rocprof trace)."""
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
    t_mut, t_tr = [], []
    for i in range(40):
        idx, s._pending_idx = s._pending_idx, None
        a = time.perf_counter()
        s.mutate(ancestors=idx)
        b = time.perf_counter()
        s._temper_reweight(with_resample=True)
        c = time.perf_counter()
        if i >= 5:
            t_mut.append(b - a)
            t_tr.append(c - b)
    torch.cuda.synchronize()
    # GPU-only time per step: the same loop, synchronised per step
    torch.cuda.synchronize()
    a = time.perf_counter()
    n = 20
    for _ in range(n):
        idx, s._pending_idx = s._pending_idx, None
        s.mutate(ancestors=idx)
        s._temper_reweight(with_resample=True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - a) / n
    # the fused step (SMCsampler._step: one launch)
    t_step = []
    for i in range(40):
        idx, s._pending_idx = s._pending_idx, None
        a = time.perf_counter()
        s._step(idx)
        if i >= 5:
            t_step.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(n):
        idx, s._pending_idx = s._pending_idx, None
        s._step(idx)
    torch.cuda.synchronize()
    wall_fused = (time.perf_counter() - a) / n
    out = {"host_mutate_us": 1e6 * sum(t_mut) / len(t_mut),
           "host_temper_reweight_us": 1e6 * sum(t_tr) / len(t_tr),
           "wall_per_step_us": 1e6 * wall,
           "host_fused_step_us": 1e6 * sum(t_step) / len(t_step),
           "wall_per_fused_step_us": 1e6 * wall_fused}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
