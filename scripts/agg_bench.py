"""Timing of the aggregation kernels: smcdet_aggregate_sweep on
joint tiles at the sizes Aggregate reaches, and the per-count-group
temper / reweight launches.  HIP-event averages over repeated launches on
synthetic populations; prints one JSON line per case.

    python scripts/agg_bench.py [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smcdet_amd.aggregate import (CountGroups, aggregate_sweep, reweight_groups,  # noqa: E402
                                  temper_groups)
from smcdet_amd.images import M71ImageModel  # noqa: E402
from smcdet_amd.kernel import SingleComponentMH  # noqa: E402
from smcdet_amd.prior import M71Prior  # noqa: E402
from tests._params import M71  # noqa: E402

DEV = "cuda"


def model(H, W):
    p = M71
    return M71ImageModel(image_height=H, image_width=W, background=p["background"],
                         psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                         psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                         noise_multiplicative=p["noise_multiplicative"])


def prior(H, W, S):
    p = M71
    return M71Prior(min_objects=0, max_objects=S, counts_rate=p["counts_rate"], image_height=H,
                    image_width=W, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                    flux_upper=p["flux_upper"], pad=4)


def population(T, N, S, H, W, smin, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    counts = torch.randint(smin, S + 1, (1, T, N), device=DEV, generator=g).float()
    counts = torch.sort(counts, -1)[0]
    pres = torch.arange(S, device=DEV) < counts[..., None]
    lo = torch.tensor([-4.0, -4.0], device=DEV)
    hi = torch.tensor([H + 4.0, W + 4.0], device=DEV)
    locs = (lo + torch.rand(1, T, N, S, 2, device=DEV, generator=g) * (hi - lo)) * pres[..., None]
    fluxes = (0.5 + 10 * torch.rand(1, T, N, S, device=DEV, generator=g)) * pres
    img = 104.0 + 10 * torch.randn(1, T, H, W, device=DEV, generator=g)
    return counts.contiguous(), locs.contiguous(), fluxes.contiguous(), img.contiguous()


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    K = 100
    for (H, W, axis, S, smin, N, T) in ((16, 8, 0, 10, 4, 4096, 2), (16, 16, 1, 20, 8, 4096, 1),
                                         (32, 32, 1, 40, 20, 4096, 1)):
        c, l, f, img = population(T, N, S, H, W, smin, 1)
        pr, mo = prior(H, W, S), model(H, W)
        mh = SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
        mh.locs_min, mh.locs_max = pr.loc_prior.low, pr.loc_prior.high
        tau = torch.full((1, T), 0.5, device=DEV)
        ws = torch.zeros(2 * T, device=DEV, dtype=torch.int32)
        ms = timed(lambda: aggregate_sweep(mo, pr, mh, axis, img, tau, c, l, f, seed=1, offset=0,
                                           acc_workspace=ws), a.reps)
        ms0 = timed(lambda: aggregate_sweep(mo, pr, mh, axis, img, tau, c, l, f, num_iters=0),
                    a.reps)
        groups = CountGroups(c)
        _, _, _, lp, lc, _ = aggregate_sweep(mo, pr, mh, axis, img, tau, c, l, f, num_iters=0)
        t0 = torch.zeros(1, T, device=DEV)
        lnc = torch.zeros(groups.G, device=DEV)
        mt = timed(lambda: temper_groups(lp * 1e-3, lc * 1e-3, t0, groups, 0.5), a.reps)
        t1 = torch.full((1, T), 0.1, device=DEV)
        mr = timed(lambda: reweight_groups(lp, lc, t1, t0, groups, lnc), a.reps)
        steps = T * N * K
        print(json.dumps(dict(
            joint=f"{H}x{W}", axis=axis, T=T, N=N, S=S, counts=f"{smin}..{S}", K=K,
            groups=groups.G, sweep_ms=ms, eval_ms=ms0,
            particle_steps_per_s=steps / ((ms - ms0) * 1e-3),
            us_per_particle_step_per_wave=(ms - ms0) * 1e3 / K,
            temper_ms=mt, reweight_ms=mr)), flush=True)


if __name__ == "__main__":
    main()
