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

Since round 5 the sweep is mh_oracle_sweep_cached (cached per-source PSF
windows; bit-identical to the full re-render in float64,
tests/test_oracle_cached.py) and two more targets exist:

  * arithmetic class "f32" (stats_<which>_oracle_f32.json): the same runs,
    same seeds and streams, in the reference's float32 arithmetic class --
    libmh_oracle_f32.so for the sweep and the log-likelihood, float32
    tempering objective and reweighting (smc_oracle dtype=float32);
  * C5 (stats_c5_oracle.json): count-stratified SMC (manuscript.tex:322-356)
    on the stats_c5.json cutout as the reference's own targets are made
    (make_golden.py gen_cssmc): for each count s = 1..6 a fixed-count run
    (S = s, N = 8192, K = 100) with its own streams (seed 1000*seed + s);
    log Z_0 = the empty catalog's log-likelihood; p(s|x) from the log Z
    vector and the reference's log p(s).

    python tests/golden/make_oracle_stats.py c2_moderate_4096_k100 <n_runs> [first_seed] [threads] [f64|f32]
    python tests/golden/make_oracle_stats.py c5 <n_runs> [first_seed] [threads]
    python tests/golden/make_oracle_stats.py queue <cycles> [threads]   # round-robin of all three
    python tests/golden/make_oracle_stats.py merge <dir>/stats_*.json    # fold in another dir's runs
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


def run_one(img, cfg, seed, threads, arith="f64"):
    H, N, S, K = cfg["tile"], cfg["N"], cfg["S"], cfg["K"]
    model = o_m71_model(H)
    prior = o_m71_prior(H, S, S, counts_rate=cfg["counts_rate"])
    mh = O.MHParams(K, 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    tiled = np.asarray(img, np.float32).reshape(1, 1, H, H)
    rng = np.random.default_rng(seed)
    rhoN = cfg["rho"] * N
    dt = np.float32 if arith == "f32" else np.float64
    # initialize (sampler.py:57-85): stratified prior draw, tau = 0, logZ = 0
    uloc = rng.random((1, 1, N, S, 2), dtype=np.float32)
    uflux = rng.random((1, 1, N, S), dtype=np.float32)
    counts, locs, fluxes = O.prior_sample_stratified(prior, 1, N, uloc, uflux)
    tau = np.zeros((1, 1), np.float32)
    logZ = np.zeros((1, 1), np.float64)
    ll = C.loglik(tiled, locs, fluxes, model, threads, arith=arith)
    tau_prev = tau
    tau, _ = O.temper(ll, tau, rhoN, dt)
    W, ess, logZ = O.update_weights(ll, tau, tau_prev, logZ, N, dt)
    esses, taus = [float(ess.flat[0])], [float(tau.flat[0])]
    it = 0
    while np.any(tau < 1) and it <= cfg["max_smc_iters"]:
        it += 1
        idx = O.systematic_resample_index(W, rng.random((1, 1), dtype=np.float32))
        counts, locs, fluxes = O.gather_particles(idx, counts, locs, fluxes)
        sweep_seed = (seed * 1000003 + it) & 0xFFFFFFFFFFFF
        locs, fluxes, _ = C.mh_sweep(tiled, counts, locs, fluxes, tau, prior, model, mh,
                                     seed=sweep_seed, threads=threads, cached=True, arith=arith)
        ll = C.loglik(tiled, locs, fluxes, model, threads, arith=arith)
        tau_prev = tau
        tau, _ = O.temper(ll, tau, rhoN, dt)
        W, ess, logZ = O.update_weights(ll, tau, tau_prev, logZ, N, dt)
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


def run_c5(ref, seed, threads, arith="f64"):
    """One CS-SMC run (manuscript.tex:322-356) of the stats_c5.json cutout:
    fixed-count runs s = 1..smax with seed 1000*seed + s (make_golden.py
    gen_cssmc's seeding), log Z_0 = the empty catalog's log-likelihood."""
    cfg = ref["config"]
    H, N, K = cfg["tile"], cfg["N"], cfg["K"]
    model = o_m71_model(H)
    tiled = np.asarray(ref["image"], np.float32).reshape(1, 1, H, H)
    ll0 = float(C.loglik(tiled, np.full((1, 1, 1, 1, 2), 4.0, np.float32),
                         np.zeros((1, 1, 1, 1), np.float32), model, 1, arith=arith).flat[0])
    lz, iters, fe, taus, hists = [ll0], [1], [float(N)], [[1.0]], [[1.0]]
    for s in range(1, cfg["smax"] + 1):
        c = dict(tile=H, N=N, S=s, K=K, rho=cfg["rho"], counts_rate=M71["counts_rate"],
                 max_smc_iters=100)
        r = run_one(ref["image"], c, 1000 * seed + s, threads, arith)
        lz.append(r["logZ"])
        iters.append(r["iters"])
        fe.append(r["final_ess"])
        taus.append(r["tau_trace"])
        hists.append(r["pruned_hist"])
    v = np.array(lz) + np.array(cfg["log_count_prior"])
    p = np.exp(v - v.max())
    return dict(seed=seed, logZ=lz, iters=iters, final_ess=fe, tau_trace=taus, pruned_hist=hists,
                count_posterior=(p / p.sum()).tolist())


def _append(out_path, cfg_out, image, row):
    doc = json.load(open(out_path)) if os.path.exists(out_path) else None
    rows = [r for r in (doc["runs"] if doc else []) if r["seed"] != row["seed"]]
    rows.append(row)
    with open(out_path + ".tmp", "w") as f:  # after every run: a partial file is usable
        json.dump(dict(config=cfg_out, image=image, runs=sorted(rows, key=lambda x: x["seed"])), f)
    os.replace(out_path + ".tmp", out_path)


def _done(out_path):
    if not os.path.exists(out_path):
        return set()
    return {r["seed"] for r in json.load(open(out_path))["runs"]}


ORACLE_DESC = {
    "f64": "oracle/mh_oracle.c (float64, cached re-render = full re-render bit for bit) + "
           "oracle/smc_oracle.py (brentq temper, softmax, systematic)",
    "f32": "oracle/mh_oracle.c -DOM_F32 (the reference's float32 arithmetic class, cached "
           "re-render) + oracle/smc_oracle.py in float32 (temper objective, reweighting)"}


# where the targets are written (SMCDET_ORACLE_OUT: e.g. gpurun_out/ on a GPU
# box, whose host cores run a batch of seeds; `merge` folds them in here)
OUT = os.environ.get("SMCDET_ORACLE_OUT", HERE)


def one_c2(which, seed, threads, arith):
    ref = json.load(open(os.path.join(HERE, f"stats_{which}.json")))
    cfg = dict(ref["config"])
    suffix = "_oracle" if arith == "f64" else "_oracle_f32"
    out_path = os.path.join(OUT, f"stats_{which}{suffix}.json")
    if seed in _done(out_path):
        return
    t0 = time.perf_counter()
    r = run_one(ref["image"], cfg, seed, threads, arith)
    r["runtime_s"] = time.perf_counter() - t0
    print(which, arith, "oracle seed", seed, round(r["logZ"], 2), r["iters"],
          f"{r['runtime_s']:.1f}s", flush=True)
    cfg_out = dict(cfg, which=f"{which}{suffix}", source="oracle", arith=arith,
                   oracle=ORACLE_DESC[arith], threads=threads)
    _append(out_path, cfg_out, ref["image"], r)


def one_c5(seed, threads, arith="f64"):
    ref = json.load(open(os.path.join(HERE, "stats_c5.json")))
    out_path = os.path.join(OUT, "stats_c5_oracle.json" if arith == "f64"
                            else "stats_c5_oracle_f32.json")
    if seed in _done(out_path):
        return
    t0 = time.perf_counter()
    r = run_c5(ref, seed, threads, arith)
    r["runtime_s"] = time.perf_counter() - t0
    print("c5", arith, "oracle seed", seed, np.round(r["logZ"][1:], 2).tolist(), r["iters"],
          f"{r['runtime_s']:.1f}s", flush=True)
    cfg_out = dict(ref["config"], which="c5_oracle", source="oracle", arith=arith,
                   oracle=ORACLE_DESC[arith], threads=threads,
                   strata="fixed-count runs s = 1..smax, seed 1000*seed + s, S = s")
    _append(out_path, cfg_out, ref["image"], r)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2_moderate_4096_k100"
    if which == "merge":
        # merge <file> ...: runs of another directory's targets into the ones here
        for src in sys.argv[2:]:
            doc = json.load(open(src))
            dst = os.path.join(HERE, os.path.basename(src))
            for r in doc["runs"]:
                _append(dst, doc["config"], doc["image"], r)
            print("merged", len(doc["runs"]), "runs of", src, "->", dst,
                  len(json.load(open(dst))["runs"]), "runs")
        return
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    if which == "queue":
        # round-robin: C5 (f64), C2 f64 (seeds 48..), C2 f32 (seeds 0..)
        threads = int(sys.argv[3]) if len(sys.argv) > 3 else 6
        for i in range(n):
            one_c5(i, threads)
            one_c2("c2_moderate_4096_k100", 48 + i, threads, "f64")
            one_c2("c2_moderate_4096_k100", i, threads, "f32")
        return
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    threads = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    arith = sys.argv[5] if len(sys.argv) > 5 else "f64"
    for seed in range(first, first + n):
        if which == "c5":
            one_c5(seed, threads, arith)
        else:
            one_c2(which, seed, threads, arith)


if __name__ == "__main__":
    main()
