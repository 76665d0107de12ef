#!/usr/bin/env python
"""CPU-baseline cross-calibration (BASELINE.md:44-46):
the reference's own SingleComponentMH (smcdet/kernel.py:26-130, torch CPU
float32, imported from /root/reference -- THIS CONTAINER ONLY, never on the
GPU box) and the C restatement bench.py times on the GPU box's host cores
(oracle/mh_oracle.c, float64 full re-render, OpenMP), on the same cores, the
same state and the same configuration: one 32x32 M71 tile (the C2 fixture
image), S = 10, N = 4096, K = 10 MH iterations at tau = 0.3 (SURVEY §6's
reference measurement).  `port_over_reference` converts the box's port figure
into a reference-equivalent one.

    python scripts/cpu_crosscal.py [threads] > profiles/r06/cpu_crosscal.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as G  # noqa: E402  (imports the reference)
from oracle import c_oracle as C  # noqa: E402
from oracle import smc_oracle as O  # noqa: E402
from tests._params import M71, o_m71_model, o_m71_prior  # noqa: E402


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.set_num_threads(threads)
    H, S, N, K, tau = 32, 10, 4096, 10, 0.3
    ref = json.load(open(os.path.join(ROOT, "tests", "golden",
                                      "stats_c2_moderate_4096_k100.json")))
    image = torch.tensor(ref["image"], dtype=torch.float32).reshape(H, H)
    torch.manual_seed(0)
    prior = G.m71_prior(H, S, S, pad=4, counts_rate=0.003125)
    mh = G.SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    s = G.sampler_for(image, H, prior, G.m71_model(H), mh, N)
    s.initialize()
    s.temperature = torch.full_like(s.temperature, tau)
    counts, locs, fluxes = (s.counts.clone(), s.locs.clone(), s.fluxes.clone())

    def ref_sweep():
        s.counts, s.locs, s.fluxes = counts.clone(), locs.clone(), fluxes.clone()
        t0 = time.perf_counter()
        s.mutate()
        return time.perf_counter() - t0

    ref_sweep()  # warm-up
    t_ref = min(ref_sweep() for _ in range(2))

    img = image.numpy().reshape(1, 1, H, H)
    c, lo, fl = (counts.numpy().astype(np.float32), locs.numpy().astype(np.float32),
                 fluxes.numpy().astype(np.float32))
    op, om = o_m71_prior(H, S, S, counts_rate=0.003125), o_m71_model(H)
    omh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    C.lib()
    out = {"config": f"{H}x{H} M71 tile (stats_c2_moderate_4096_k100 image), S={S}, N={N}, "
                     f"K={K} MH iterations at tau={tau}", "threads": threads,
           "host": f"{os.cpu_count()} CPUs visible"}
    out["reference"] = {"seconds": t_ref, "particle_steps_per_s": N * K / t_ref,
                        "what": "reference SMCsampler.mutate() -> SingleComponentMH.run "
                                "(smcdet/kernel.py:26-130), torch CPU float32, "
                                f"torch.set_num_threads({threads})"}
    for key, kw in (("port", dict(cached=False)), ("port_cached", dict(cached=True)),
                    ("port_cached_f32", dict(cached=True, arith="f32"))):
        C.mh_sweep(img, c, lo, fl, tau, op, om, omh, seed=1, threads=threads, **kw)  # warm-up
        ts = []
        for rep in range(2):
            t0 = time.perf_counter()
            C.mh_sweep(img, c, lo, fl, tau, op, om, omh, seed=2 + rep, threads=threads, **kw)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        out[key] = {"seconds": t, "particle_steps_per_s": N * K / t,
                    "port_over_reference": (N * K / t) / (N * K / t_ref)}
    out["port"]["what"] = ("oracle/mh_oracle.c float64 full re-render (bench.py cpu_baseline's "
                           "kernel), OpenMP")
    out["port_cached"]["what"] = "the same with cached per-source PSF windows (bit-identical)"
    out["port_cached_f32"]["what"] = "the float32-class build (-DOM_F32), cached"
    out["port_over_reference"] = out["port"]["port_over_reference"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
