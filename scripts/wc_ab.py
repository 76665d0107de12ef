#!/usr/bin/env python
"""A/B of the MH sweep with and without the PSF window cache at the C2
geometry: bit-equality of the outputs (same draws), then interleaved timing.

    python scripts/wc_ab.py [--rounds 7] [--tau 0.3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from smcdet_amd._rng import PhiloxStream  # noqa: E402
from tests._params import GOLDEN, M71, p_m71_mh, p_m71_model, p_m71_prior  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--tau", type=float, default=0.3)
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--particles", type=int, default=4096)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    H, S, Np = 32, 10, a.particles
    model, prior = p_m71_model(H), p_m71_prior(H, S, S, counts_rate=0.003125)
    ref = json.load(open(os.path.join(GOLDEN, "stats_c2_moderate.json")))
    img = torch.tensor(ref["image"], dtype=torch.float32).reshape(1, 1, H, H).to(dev)
    g = torch.Generator().manual_seed(1)
    counts = torch.full((1, 1, Np), float(S), device=dev)
    locs = (torch.rand(1, 1, Np, S, 2, generator=g) * (H + 8) - 4).to(dev)
    al, lo, hi = M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"]
    u = torch.rand(1, 1, Np, S, generator=g, dtype=torch.float64)
    fl = ((hi ** al - u * hi ** al + u * lo ** al) / (lo ** al * hi ** al)) ** (-1 / al)
    fluxes = fl.float().clamp(lo, hi).to(dev)
    tau = torch.full((1, 1), a.tau, device=dev)
    mw = p_m71_mh(a.K)
    mw.rng = PhiloxStream(123)
    for _ in range(3):
        locs, fluxes, _ = mw.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model)
    r_in = torch.empty(1, 1, Np, H * H, device=dev)
    p_m71_mh(0).run(img, counts, locs, fluxes, tau, prior=prior, image_model=model, rate_out=r_in)

    def sweep(wc, seed=7):
        mh = p_m71_mh(a.K)
        mh.psf_cache = wc
        mh.rng = PhiloxStream(seed)
        r_out = torch.empty_like(r_in)
        out = mh.run(img, counts, locs, fluxes, tau, prior=prior, image_model=model,
                     rate_in=r_in, rate_out=r_out)
        return out, r_out, mh

    res = {}
    (l0, f0, a0), r0, m0 = sweep(False)
    (l1, f1, a1), r1, m1 = sweep(True)
    torch.cuda.synchronize()
    res["equal"] = {"locs": bool(torch.equal(l0, l1)), "fluxes": bool(torch.equal(f0, f1)),
                    "loglik": bool(torch.equal(m0.last_loglik, m1.last_loglik)),
                    "rate_out": bool(torch.equal(r0, r1)),
                    "acc_rate": [float(a0.flatten()[0]), float(a1.flatten()[0])]}
    res["moved_fraction"] = float((l0 != locs).any(-1).float().mean())
    print(json.dumps(res), flush=True)

    REP = 5
    times = {"base": [], "wcache": []}
    for r in range(a.rounds + 1):
        for k in times:
            mh = p_m71_mh(a.K)
            mh.psf_cache = k == "wcache"
            mh.rng = PhiloxStream(11)
            r_out = torch.empty_like(r_in)
            fn = lambda: mh.run(img, counts, locs, fluxes, tau, prior=prior,  # noqa: E731
                                image_model=model, rate_in=r_in, rate_out=r_out)
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REP):
                fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[k].append(e0.elapsed_time(e1) / REP)
    res["ms"] = {k: {"median": float(np.median(v)), "min": float(np.min(v)), "all": v}
                 for k, v in times.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
