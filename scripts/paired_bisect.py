#!/usr/bin/env python
"""Bisects where a paired GPU run (tests/test_gpu_paired.py: the oracle's
own draws replayed on the GPU) leaves its oracle twin: per seed and variant,
the temperature and log Z after every SMC iteration, next to the oracle run's
recorded ladder (tests/golden/stats_c2_moderate_4096_k100_oracle.json).

Variants (same draws throughout):
  gpu         the paired test's schedule (incremental MH, ancestors gathered
              in the sweep, device temper / reweight / systematic indices)
  gpu_full    the same with full re-render MH steps (the reference's float32
              arithmetic per step: SingleComponentMH(full_recompute=True))
  oracle_tile GPU sweeps, but temper / update_weights / resampling indices by
              the oracle (float64 C log-likelihoods of the GPU population,
              brentq, softmax, bucketize) -- isolates the tile pass
  oracle_init the gpu variant started from the oracle's own prior draw

    python scripts/paired_bisect.py --seeds 12 24 40 43 0 4 --out gpurun_out/bisect.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import c_oracle as C  # noqa: E402
from oracle import smc_oracle as O  # noqa: E402
from tests._params import (GOLDEN, M71, o_m71_model, p_m71_mh, p_m71_model,  # noqa: E402
                           p_m71_prior)

DEV = torch.device("cuda", 0)


def run(img, cfg, seed, variant, threads):
    from smcdet_amd.sampler import SMCsampler
    H, N, S, K = cfg["tile"], cfg["N"], cfg["S"], cfg["K"]
    prior = p_m71_prior(H, S, S, counts_rate=cfg["counts_rate"])
    model = p_m71_model(H)
    mh = p_m71_mh(K, full_recompute=(variant == "gpu_full"))
    image = torch.tensor(img, dtype=torch.float32, device=DEV)
    s = SMCsampler(image, H, prior, model, mh, N, cfg["rho"], "systematic",
                   M71["flux_detection_threshold"], cfg["max_smc_iters"], print_every=10 ** 9,
                   device=DEV)
    rng = np.random.default_rng(seed)
    uloc = rng.random((1, 1, N, S, 2), dtype=np.float32)
    uflux = rng.random((1, 1, N, S), dtype=np.float32)
    if variant == "oracle_init":
        from tests._params import o_m71_prior
        op = o_m71_prior(H, S, S, counts_rate=cfg["counts_rate"])
        c, l, f = O.prior_sample_stratified(op, 1, N, uloc, uflux)
        s.counts, s.locs, s.fluxes = (torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(DEV)
                                      for x in (c, l, f))
    else:
        s.counts, s.locs, s.fluxes = prior.sample_stratified(
            1, N, device=DEV, uloc=torch.from_numpy(uloc).to(DEV),
            uflux=torch.from_numpy(uflux).to(DEV))
    om = o_m71_model(H)
    tiled = np.asarray(img, np.float32).reshape(1, 1, H, H)
    rho_n = cfg["rho"] * N
    s.temperature_prev = torch.zeros(1, 1, device=DEV)
    s.temperature = torch.zeros(1, 1, device=DEV)
    s.log_normalizing_constant = torch.zeros(1, 1, device=DEV)
    s._fresh_loglik = None
    host = variant == "oracle_tile"
    if host:
        tau = np.zeros((1, 1), np.float32)
        lz = np.zeros((1, 1), np.float64)
        ll = C.loglik(tiled, s.locs.cpu().numpy(), s.fluxes.cpu().numpy(), om, threads)
        tau_prev = tau
        tau, _ = O.temper(ll, tau, rho_n)
        W, ess, lz = O.update_weights(ll, tau, tau_prev, lz, N)
    else:
        s.temper()
        s.update_weights()
    taus, lzs, it = [], [], 0
    while True:
        t_now = float(tau.flat[0]) if host else float(s.temperature.flatten()[0])
        taus.append(t_now)
        lzs.append(float(lz.flat[0]) if host else float(s.log_normalizing_constant.flatten()[0]))
        if t_now >= 1.0 or it > cfg["max_smc_iters"]:
            break
        it += 1
        u = rng.random((1, 1), dtype=np.float32)
        if host:
            idx = torch.from_numpy(O.systematic_resample_index(W, u).astype(np.int64)).to(DEV)
        else:
            idx = s.resample_index(u=torch.from_numpy(u).to(DEV))
        d = C.sweep_draws((seed * 1000003 + it) & 0xFFFFFFFFFFFF, 1, N, K, S)
        replay = {k: torch.from_numpy(v.reshape((K, 1, 1) + v.shape[2:])) for k, v in d.items()}
        if host:
            s.temperature = torch.from_numpy(np.asarray(tau, np.float32)).to(DEV)
        s.locs, s.fluxes, s.mutation_acc_rates = mh.run(
            s.tiled_image, s.counts, s.locs, s.fluxes, s.temperature, s.log_target,
            ancestors=idx.reshape(1, 1, N).contiguous(), replay=replay)
        s.counts = mh.last_counts
        if host:
            ll = C.loglik(tiled, s.locs.cpu().numpy(), s.fluxes.cpu().numpy(), om, threads)
            tau_prev = tau
            tau, _ = O.temper(ll, tau, rho_n)
            W, ess, lz = O.update_weights(ll, tau, tau_prev, lz, N)
        else:
            s._fresh_loglik = mh.last_loglik
            s.temper()
            s.update_weights()
    return dict(seed=seed, variant=variant, iters=it, logZ=lzs[-1], tau=taus, logZ_trace=lzs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[12, 24, 40, 43, 0, 4, 8, 16])
    ap.add_argument("--variants", nargs="+",
                    default=["gpu", "gpu_full", "oracle_tile", "oracle_init"])
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/paired_bisect.json")
    a = ap.parse_args()
    ref = json.load(open(os.path.join(GOLDEN, "stats_c2_moderate_4096_k100_oracle.json")))
    runs = {r["seed"]: r for r in ref["runs"]}
    out = []
    for seed in a.seeds:
        r = runs[seed]
        row = {"seed": seed, "oracle": {"logZ": r["logZ"], "iters": r["iters"],
                                        "tau": r["tau_trace"]}}
        for v in a.variants:
            t0 = time.perf_counter()
            x = run(ref["image"], ref["config"], seed, v, a.threads)
            # first iteration whose temperature leaves the oracle's ladder
            ot = r["tau_trace"]
            n = min(len(ot), len(x["tau"]))
            dev = [i for i in range(n) if abs(ot[i] - x["tau"][i]) > 1e-5]
            x["first_tau_divergence"] = dev[0] if dev else None
            x["seconds"] = time.perf_counter() - t0
            row[v] = x
            print(f"seed {seed} {v}: log Z {x['logZ']:.2f} ({x['iters']} it) vs oracle "
                  f"{r['logZ']:.2f} ({r['iters']} it); tau leaves the oracle ladder at "
                  f"iteration {x['first_tau_divergence']}", flush=True)
        out.append(row)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
