#!/usr/bin/env python
"""north_star's "log Z and ESS within 1%" at the headline configuration,
resolved by sample size: n independent GPU runs of SMCsampler at C2 (one
32x32 M71 tile -- the stats_c2_moderate_4096_k100 image --, S = 10, N = 4096,
K = 100, systematic, rho = 0.5; one launch grid of n copies of the tile,
independent stopping) against every run of the float64 oracle target
(tests/golden/stats_c2_moderate_4096_k100_oracle.json) and the reference's own
runs: mean log Z, mean final ESS (the ESS of each run's last reweighting,
sampler.py:181-196), SMC iterations, the lower log Z mode's share, and the
count posterior (tests/_stats.py).  Each mean difference is reported
relative to the target mean and in pooled standard errors, with the 95%
interval of the relative difference -- "within 1%" is resolved when that
interval lies inside +-1%.

    python scripts/c2_law.py [n_runs=8192] > profiles/r06/c2_law.json

SMCDET_LAW_DUMP=<file.npz> also writes the GPU runs' per-run summaries
(log Z, final ESS, iterations, pruned-count histogram, pruned flux), so the
comparison can be recomputed on the CPU against a grown target without
another GPU run:

    python scripts/c2_law.py --recompute <file.npz> > profiles/r06/c2_law.json
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

from tests._stats import count_posterior_compare, hist_var  # noqa: E402


def gpu_runs(ref, n_runs, seed, chunk=2048):
    import bench
    from smcdet_amd.images import M71ImageModel
    from smcdet_amd.kernel import SingleComponentMH
    from smcdet_amd.prior import M71Prior
    from smcdet_amd.sampler import SMCsampler
    dev = torch.device("cuda", 0)
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
    runs = []
    for c0 in range(0, n_runs, chunk):
        n = min(chunk, n_runs - c0)
        tiles = img.reshape(1, 1, H, H).expand(1, n, H, H).contiguous()
        mh = SingleComponentMH(K, 0.1, 2.5, p["flux_lower"], p["flux_upper"])
        s = SMCsampler.from_tiles(tiles, prior, model, mh, N, cfg["rho"], cfg["method"],
                                  p["flux_detection_threshold"], cfg.get("max_smc_iters", 1000),
                                  print_every=10 ** 9, seed=seed + c0, device=dev,
                                  stopping="independent")
        with contextlib.redirect_stdout(io.StringIO()):
            s.run()
        lz = s.log_normalizing_constant.reshape(-1).double().cpu().numpy()
        fe = s.ess.reshape(-1).double().cpu().numpy()
        it = s.iters_per_tile.reshape(-1).cpu().numpy()
        pc = s.pruned_counts.reshape(n, -1)
        hists = torch.stack([torch.bincount(pc[i], minlength=S + 1)[:S + 1] for i in range(n)])
        hists = (hists.double() / pc.shape[-1]).cpu().numpy()
        pflux = s.posterior_mean_total_flux(s.pruned_fluxes).reshape(-1).double().cpu().numpy()
        for i in range(n):
            runs.append({"logZ": float(lz[i]), "final_ess": float(fe[i]), "iters": int(it[i]),
                         "pruned_hist": hists[i].tolist(),
                         "mean_total_flux_pruned": float(pflux[i])})
        del s
        torch.cuda.empty_cache()
        print(f"{c0 + n} runs", file=sys.stderr, flush=True)  # progress
    return runs


def compare(ours, theirs, key):
    a = np.array([r[key] for r in ours], dtype=np.float64)
    b = np.array([r[key] for r in theirs], dtype=np.float64)
    se = float(np.sqrt(a.var(ddof=1) / a.size + b.var(ddof=1) / b.size))
    d = float(a.mean() - b.mean())
    rel, rel_se = d / abs(b.mean()), se / abs(b.mean())
    return {"ours": float(a.mean()), "target": float(b.mean()), "n": [int(a.size), int(b.size)],
            "sd": [float(a.std(ddof=1)), float(b.std(ddof=1))], "rel_diff": rel,
            "rel_diff_95": [rel - 1.96 * rel_se, rel + 1.96 * rel_se],
            "within_1pct_resolved": bool(abs(rel) + 1.96 * rel_se < 0.01),
            "diff_in_pooled_se": d / se if se > 0 else 0.0}


def dump(runs, path, meta):
    np.savez_compressed(
        path, logZ=np.array([r["logZ"] for r in runs]),
        final_ess=np.array([r["final_ess"] for r in runs]),
        iters=np.array([r["iters"] for r in runs], dtype=np.int32),
        pruned_hist=np.array([r["pruned_hist"] for r in runs], dtype=np.float64),
        mean_total_flux_pruned=np.array([r["mean_total_flux_pruned"] for r in runs]),
        meta=json.dumps(meta))


def load(path):
    z = np.load(path, allow_pickle=False)
    runs = [{"logZ": float(a), "final_ess": float(b), "iters": int(c), "pruned_hist": h.tolist(),
             "mean_total_flux_pruned": float(f)}
            for a, b, c, h, f in zip(z["logZ"], z["final_ess"], z["iters"], z["pruned_hist"],
                                     z["mean_total_flux_pruned"])]
    return runs, json.loads(str(z["meta"]))


def main():
    g = os.path.join(ROOT, "tests", "golden")
    orc = json.load(open(os.path.join(g, "stats_c2_moderate_4096_k100_oracle.json")))
    ref = json.load(open(os.path.join(g, "stats_c2_moderate_4096_k100.json")))
    if len(sys.argv) > 2 and sys.argv[1] == "--recompute":
        ours, out = load(sys.argv[2])
        out["recomputed_from"] = os.path.basename(sys.argv[2])
    else:
        n_runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
        t0 = time.perf_counter()
        ours = gpu_runs(ref, n_runs, seed=90210)
        out = {"config": "C2: 32x32 M71 tile (stats_c2_moderate_4096_k100 image), S=10, N=4096, "
                         "K=100, systematic, rho=0.5; GPU runs = one launch grid of copies, "
                         "independent stopping",
               "gpu_runs": len(ours), "gpu_wall_s": time.perf_counter() - t0,
               "library": __import__("smcdet_amd._hip", fromlist=["x"]).version()}
        if os.environ.get("SMCDET_LAW_DUMP"):
            dump(ours, os.environ["SMCDET_LAW_DUMP"], out)
    out["oracle_runs"] = len(orc["runs"])
    cut = float(np.median([r["logZ"] for r in orc["runs"]]) - 40.0)
    for name, tgt in (("vs_oracle", orc["runs"]), ("vs_reference", ref["runs"])):
        res = {k: compare(ours, tgt, k) for k in ("logZ", "final_ess", "iters")}
        lo_a = float(np.mean([r["logZ"] < cut for r in ours]))
        lo_b = float(np.mean([r["logZ"] < cut for r in tgt]))
        res["lower_mode_share"] = {"cut": cut, "ours": lo_a, "target": lo_b}
        res["count_posterior"] = count_posterior_compare(
            ours, tgt, var_floor=hist_var(orc["runs"]) if name == "vs_reference" else None)
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
