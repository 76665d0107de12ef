#!/usr/bin/env python
"""Fixed cost of a timed region (C2): bench.py times K steps between two
synchronisations, so ms_per_step = GPU step + C/K.  Measures the wall time
of K = 1..40 back-to-back SMC steps, the host time to enqueue the first step
after a synchronisation, and an idle synchronisation, to split C into host
enqueue and the rest."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
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
    out = {"wall_ms": {}, "first_enqueue_us": [], "idle_sync_us": []}
    for k in (1, 2, 5, 10, 20, 40, 1, 2, 5, 10, 20, 40):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        for _ in range(k - 1):
            step()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out["wall_ms"].setdefault(k, []).append((t2 - t0) * 1e3)
        out["first_enqueue_us"].append((t1 - t0) * 1e6)
        a = time.perf_counter()
        torch.cuda.synchronize()
        out["idle_sync_us"].append((time.perf_counter() - a) * 1e6)
        print(k, round((t2 - t0) * 1e3 / k, 4), "ms/step", flush=True)
    ks = np.array(sorted(out["wall_ms"]), dtype=np.float64)
    w = np.array([min(out["wall_ms"][int(k)]) for k in ks])
    slope, icpt = np.polyfit(ks, w, 1)
    out["fit"] = {"gpu_ms_per_step": slope, "fixed_ms": icpt}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
