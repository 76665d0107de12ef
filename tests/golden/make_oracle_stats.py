#!/usr/bin/env python
"""Statistical targets from the ORACLE (test infrastructure): complete
SMCsampler.run()s of the reference's algorithm (smcdet/sampler.py:221-256;
resample -> mutate -> temper -> update_weights) restated on the CPU --
the float64 C MH sweep of oracle/mh_oracle.c with full re-renders
(smcdet/kernel.py:26-130), brentq tempering, softmax reweighting and
systematic resampling of oracle/smc_oracle.py -- with their own random
streams (numpy PCG64 for the prior draw and resampling offsets, splitmix64
per particle and SMC iteration inside the sweep).

The reference itself takes ~75 min per run at the headline configuration
(N=4096, K=100) on 2 cores, so it contributes few seeds
(stats_c2_moderate_4096_k100.json); the oracle takes ~1 min per run on 8,
which resolves the tails of the log Z distribution (e.g. how often a run
settles in the lower mode) that a handful of reference seeds cannot.  The
rows have the format of make_golden.py gen_stats, so
tests/test_gpu_statistical.py reads them the same way.

    python tests/golden/make_oracle_stats.py c2_moderate_4096_k100 <n_runs> [first_seed] [threads]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import c_oracle as C  # noqa: E402
from oracle import smc_oracle as O  # noqa: E402
from tests._params import M71, o_m71_model, o_m71_prior  # noqa: E402


def run_one(img, cfg, seed, threads):
    H, N, S, K = cfg["tile"], cfg["N"], cfg["S"], cfg["K"]
    model = o_m71_model(H)
    prior = o_m71_prior(H, S, S, counts_rate=cfg["counts_rate"])
    mh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    tiled = np.asarray(img, np.float32).reshape(1, 1, H, H)
    rng = np.random.default_rng(seed)
    rhoN = cfg["rho"] * N
    # initialize (sampler.py:57-85): stratified prior draw, tau = 0, logZ = 0
    uloc = rng.random((1, 1, N, S, 2), dtype=np.float32)
    uflux = rng.random((1, 1, N, S), dtype=np.float32)
    counts, locs, fluxes = O.prior_sample_stratified(prior, 1, N, uloc, uflux)
    tau = np.zeros((1, 1), np.float32)
    logZ = np.zeros((1, 1), np.float64)
    ll = C.loglik(tiled, locs, fluxes, model, threads)
    tau_prev = tau
    tau, _ = O.temper(ll, tau, rhoN)
    W, ess, logZ = O.update_weights(ll, tau, tau_prev, logZ, N)
    esses, taus = [float(ess.flat[0])], [float(tau.flat[0])]
    it = 0
    while np.any(tau < 1) and it <= cfg["max_smc_iters"]:
        it += 1
        idx = O.systematic_resample_index(W, rng.random((1, 1), dtype=np.float32))
        counts, locs, fluxes = O.gather_particles(idx, counts, locs, fluxes)
        sweep_seed = (seed * 1000003 + it) & 0xFFFFFFFFFFFF
        locs, fluxes, _ = C.mh_sweep(tiled, counts, locs, fluxes, tau, prior, model, mh,
                                     seed=sweep_seed, threads=threads)
        ll = C.loglik(tiled, locs, fluxes, model, threads)
        tau_prev = tau
        tau, _ = O.temper(ll, tau, rhoN)
        W, ess, logZ = O.update_weights(ll, tau, tau_prev, logZ, N)
        esses.append(float(ess.flat[0]))
        taus.append(float(tau.flat[0]))
    final_ess = float(ess.flat[0])
    idx = O.systematic_resample_index(W, rng.random((1, 1), dtype=np.float32))
    counts, locs, fluxes = O.gather_particles(idx, counts, locs, fluxes)
    pc, pl, pf = O.prune(locs, fluxes, H, M71["flux_detection_threshold"])
    hist = np.bincount(pc.reshape(-1).astype(np.int64), minlength=S + 1)
    return dict(seed=seed, logZ=float(logZ.flat[0]), iters=it, ess_trace=esses, tau_trace=taus,
                final_ess=final_ess, pruned_hist=(hist / hist.sum()).tolist(),
                mean_total_flux=float(fluxes.sum(-1).mean()),
                mean_total_flux_pruned=float(pf.sum(-1).mean()))


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2_moderate_4096_k100"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    threads = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    ref = json.load(open(os.path.join(HERE, f"stats_{which}.json")))
    cfg = dict(ref["config"])
    out_path = os.path.join(HERE, f"stats_{which}_oracle.json")
    doc = json.load(open(out_path)) if os.path.exists(out_path) else None
    rows = doc["runs"] if doc else []
    done = {r["seed"] for r in rows}
    for seed in range(first, first + n):
        if seed in done:
            continue
        t0 = time.perf_counter()
        r = run_one(ref["image"], cfg, seed, threads)
        r["runtime_s"] = time.perf_counter() - t0
        rows.append(r)
        print(which, "oracle seed", seed, round(r["logZ"], 2), r["iters"],
              f"{r['runtime_s']:.1f}s", flush=True)
        cfg_out = dict(cfg, which=f"{which}_oracle", source="oracle",
                       oracle="oracle/mh_oracle.c (float64, full re-render) + "
                              "oracle/smc_oracle.py (brentq temper, softmax, systematic)",
                       threads=threads)
        with open(out_path, "w") as f:  # after every run: a partial file is usable
            json.dump(dict(config=cfg_out, image=ref["image"],
                           runs=sorted(rows, key=lambda x: x["seed"])), f)
    print("wrote", out_path, len(rows), "runs")


if __name__ == "__main__":
    main()
