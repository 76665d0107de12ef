#!/usr/bin/env python
"""Diagnostic: the log Z distribution of many independent C2-configuration
runs (one launch grid of copies of the tile, independent stopping) under
sampler variants, to locate where a lower log Z mode comes from: default,
persisted rate images off, full re-render MH (the reference's arithmetic per
step), the unfused loop.  Prints one JSON line per variant: mean, sd,
quantiles, the share below a cut, and iteration counts.

    python scripts/logz_modes.py [which=c2_moderate_4096_k100] [n_runs=256] [variants=all] [cut]
"""
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smcdet_amd.images import M71ImageModel  # noqa: E402
from smcdet_amd.kernel import SingleComponentMH  # noqa: E402
from smcdet_amd.prior import M71Prior  # noqa: E402
from smcdet_amd.sampler import SMCsampler  # noqa: E402

VARIANTS = {
    "default": {},
    "no_persist": {"persist_rate_images": False},
    "full": {"full_recompute": True},
    "unfused": {"fused": False, "stopping": "lockstep"},
    "refresh1": {"rate_refresh_every": 1},
    # the MH sweep's per-pixel form everywhere (SMCDET_MH_NO_BLOCK): the
    # block form's profile rounding vs the per-pixel one's
    "no_block": {"debug_flags": 16384},
}


def run(which, n_runs, variant, seed=777):
    dev = torch.device("cuda", 0)
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", f"stats_{which}.json")))
    cfg = ref["config"]
    p, H, S, N, K = bench.M71, cfg["tile"], cfg["S"], cfg["N"], cfg["K"]
    model = M71ImageModel(image_height=H, image_width=H, background=p["background"],
                          psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])
    prior = M71Prior(min_objects=S, max_objects=S, counts_rate=cfg["counts_rate"],
                     image_height=H, image_width=H, flux_alpha=p["flux_alpha"],
                     flux_lower=p["flux_lower"], flux_upper=p["flux_upper"], pad=4)
    img = torch.tensor(ref["image"], dtype=torch.float32, device=dev)
    tiles = img.reshape(1, 1, H, H).expand(1, n_runs, H, H).contiguous()
    v = dict(VARIANTS[variant])
    mh = SingleComponentMH(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"],
                           full_recompute=v.pop("full_recompute", False))
    mh.debug_flags = v.pop("debug_flags", 0)
    s = SMCsampler.from_tiles(tiles, prior, model, mh, N, cfg["rho"], cfg["method"],
                              p["flux_detection_threshold"], cfg.get("max_smc_iters", 1000),
                              print_every=10 ** 9, seed=seed, device=dev,
                              **dict({"stopping": "independent"}, **v))
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        s.run()
    torch.cuda.synchronize()
    return (s.log_normalizing_constant.flatten().double().cpu().numpy(),
            s.iters_per_tile.flatten().double().cpu().numpy(), time.perf_counter() - t0)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2_moderate_4096_k100"
    n_runs = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    names = sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] != "all" else list(VARIANTS)
    cut = float(sys.argv[4]) if len(sys.argv) > 4 else -4310.0
    for name in names:
        lz, it, wall = run(which, n_runs, name)
        print(json.dumps({"variant": name, "n": n_runs, "wall_s": round(wall, 2),
                          "logZ_mean": float(lz.mean()), "logZ_sd": float(lz.std(ddof=1)),
                          "logZ_q": np.percentile(lz, [0, 5, 10, 25, 50, 75, 100]).round(1).tolist(),
                          "share_below_cut": float((lz < cut).mean()), "cut": cut,
                          "iters_mean": float(it.mean()), "iters_sd": float(it.std(ddof=1)),
                          "iters_low_mode": float(it[lz < cut].mean()) if (lz < cut).any() else None}),
              flush=True)


if __name__ == "__main__":
    main()
