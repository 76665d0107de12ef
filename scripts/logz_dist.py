#!/usr/bin/env python
"""Distribution of log Z (and iterations, final ESS) over many runs of this
sampler at a recorded reference configuration (tests/golden/stats_<which>.json),
next to the reference's own runs: quantiles, and how many of ours fall below
the reference's lowest run.  Uses bench.vs_reference's setup (one launch grid
of independent copies of the tile, independent stopping).

    python scripts/logz_dist.py [which=c2_moderate_4096_k100] [n_runs=256] [seed]
"""
import contextlib
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smcdet_amd.images import M71ImageModel  # noqa: E402
from smcdet_amd.kernel import SingleComponentMH  # noqa: E402
from smcdet_amd.prior import M71Prior  # noqa: E402
from smcdet_amd.sampler import SMCsampler  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2_moderate_4096_k100"
    n_runs = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 777
    dev = torch.device("cuda", 0)
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", f"stats_{which}.json")))
    cfg, rr = ref["config"], ref["runs"]
    p, H, S, N, K = bench.M71, cfg["tile"], cfg["S"], cfg["N"], cfg["K"]
    model = M71ImageModel(image_height=H, image_width=H, background=p["background"],
                          psf_radius=p["psf_radius"], adu_per_nmgy=p["adu_per_nmgy"],
                          psf_params=p["psf_params"], noise_additive=p["noise_additive"],
                          noise_multiplicative=p["noise_multiplicative"])
    prior = M71Prior(min_objects=S, max_objects=S, counts_rate=bench.COUNTS_RATE_C2,
                     image_height=H, image_width=H, flux_alpha=p["flux_alpha"],
                     flux_lower=p["flux_lower"], flux_upper=p["flux_upper"], pad=4)
    img = torch.tensor(ref["image"], dtype=torch.float32, device=dev)
    tiles = img.reshape(1, 1, H, H).expand(1, n_runs, H, H).contiguous()
    mh = SingleComponentMH(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])
    s = SMCsampler.from_tiles(tiles, prior, model, mh, N, cfg["rho"], cfg["method"],
                              p["flux_detection_threshold"], cfg.get("max_smc_iters", 1000),
                              print_every=10 ** 9, seed=seed, device=dev,
                              stopping="independent")
    with contextlib.redirect_stdout(io.StringIO()):
        s.run()
    ours = {"logZ": s.log_normalizing_constant.flatten().double().cpu().numpy(),
            "iters": s.iters_per_tile.flatten().double().cpu().numpy(),
            "final_ess": s.ess.flatten().double().cpu().numpy()}
    theirs = {k: np.array([r[k] for r in rr], dtype=np.float64) for k in ours}
    q = [0, 5, 10, 25, 50, 75, 90, 95, 100]
    out = {"which": which, "n_ours": n_runs, "n_reference": len(rr), "seed": seed}
    for k in ours:
        a, b = ours[k], theirs[k]
        out[k] = {"ours_q": np.percentile(a, q).round(2).tolist(),
                  "reference_q": np.percentile(b, q).round(2).tolist(),
                  "ours_mean_sd": [float(a.mean()), float(a.std(ddof=1))],
                  "reference_mean_sd": [float(b.mean()), float(b.std(ddof=1))],
                  "ours_below_reference_min": float((a < b.min()).mean()),
                  "ours_above_reference_max": float((a > b.max()).mean())}
    out["ours_logZ_sorted"] = np.sort(ours["logZ"]).round(1).tolist()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
