#!/usr/bin/env python
"""cProfile of the host side of SMCsampler._step at C2 (bench.py's step):
which Python calls the per-step enqueue time goes to."""
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
    n = 30
    t = []
    for _ in range(n):
        a = time.perf_counter()
        step()
        t.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    t.sort()
    print(f"host enqueue per step: median {1e6 * t[n // 2]:.1f} us, min {1e6 * t[0]:.1f} us",
          flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        step()
    pr.disable()
    torch.cuda.synchronize()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(40)
    print(out.getvalue())


if __name__ == "__main__":
    main()
