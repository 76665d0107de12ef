"""Aggregate vs single-tile sampler on the same image.

Runs count-stratified SMC on the 2x2 8x8 tiles of the 16x16 fixture image
(tests/golden/agg_m71_pieces.npz), aggregates them (smcdet_amd.aggregate),
and count-stratified SMC on the whole 16x16 tile, at several particle / MH
budgets; prints one JSON line per run with the posterior mean number of
detectable stars in the image, their total flux, log evidence and wall time.

    python scripts/agg_validate.py [--seeds 3] [--configs 512x50,2048x100,...]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smcdet_amd.aggregate import Aggregate  # noqa: E402
from smcdet_amd.cssmc import CountStratifiedSMC  # noqa: E402
from smcdet_amd.images import M71ImageModel  # noqa: E402
from smcdet_amd.kernel import SingleComponentMH  # noqa: E402
from smcdet_amd.prior import M71Prior  # noqa: E402
from tests._params import M71, golden  # noqa: E402


def model(H):
    p = M71
    return M71ImageModel(image_height=H, image_width=H, background=p["background"],
                         psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                         psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                         noise_multiplicative=p["noise_multiplicative"])


def prior(H, smax, rate, pad):
    p = M71
    return M71Prior(min_objects=0, max_objects=smax, counts_rate=rate, image_height=H,
                    image_width=H, flux_alpha=p["flux_alpha"], flux_lower=p["flux_lower"],
                    flux_upper=p["flux_upper"], pad=pad)


def mh(K):
    return SingleComponentMH(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])


def quiet(fn):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn()


def summary(counts, fluxes):
    return float(counts.float().mean()), float(fluxes.sum(-1).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--configs", default="512x50,2048x100,4096x200")
    ap.add_argument("--rate", type=float, default=0.01)
    ap.add_argument("--pad", type=int, default=2)
    ap.add_argument("--image", default="agg")
    a = ap.parse_args()
    if a.image == "agg":  # two of the five stars within 0.4 px of a tile boundary
        img = torch.as_tensor(golden("agg_m71_pieces.npz")["image"], device="cuda")
    else:  # "centred": four stars near the centres of the four 8x8 tiles
        torch.manual_seed(17)
        l = torch.tensor([[[[[3.5, 4.2], [4.1, 11.6], [12.3, 3.8], [11.7, 12.2]]]]], device="cuda")
        f = torch.tensor([[[[6.0, 4.0, 3.0, 5.0]]]], device="cuda")
        img = model(16).sample(l, f)[0, 0, :, :, 0]
    thr = M71["flux_detection_threshold"]
    for cfg in a.configs.split(","):
        N, K = (int(x) for x in cfg.split("x"))
        for seed in range(a.seeds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            kids = CountStratifiedSMC(img, 8, prior(8, 6, a.rate, a.pad), model(8), mh(K), N, 0.5,
                                      "systematic", thr, 200, print_every=10 ** 9,
                                      num_catalogs=N, seed=100 + seed)
            quiet(kids.run)
            agg = Aggregate(prior(8, 6, a.rate, a.pad), model(8), mh(K), kids.tiled_image,
                            kids.counts, kids.locs, kids.fluxes, kids.weights,
                            kids.log_normalizing_constant, thr, "systematic", 0.5,
                            print_every=10 ** 9, seed=200 + seed)
            quiet(agg.run)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            big = CountStratifiedSMC(img, 16, prior(16, 12, a.rate, a.pad), model(16), mh(K), N,
                                     0.5, "systematic", thr, 200, print_every=10 ** 9,
                                     num_catalogs=N, seed=300 + seed)
            quiet(big.run)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            ac, af = summary(agg.pruned_counts, agg.pruned_fluxes)
            bc, bf = summary(big.pruned_counts, big.pruned_fluxes)
            print(json.dumps(dict(
                image=a.image, N=N, K=K, seed=seed, agg_count=ac, big_count=bc, agg_flux=af, big_flux=bf,
                agg_lz=float(agg.log_evidence.reshape(-1)[0]),
                kids_lz=kids.log_normalizing_constant.reshape(-1).tolist(),
                big_lz=float(big.log_normalizing_constant.reshape(-1)[0]),
                agg_iters=agg.iters_per_level, big_iters=int(big.iter),
                agg_S=int(agg.locs.shape[-2]),
                big_count_post=big.count_posterior.reshape(-1).tolist(),
                t_agg=t1 - t0, t_big=t2 - t1)), flush=True)


if __name__ == "__main__":
    main()
