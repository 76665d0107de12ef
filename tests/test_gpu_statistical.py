"""Statistical parity of whole SMC runs against the reference.

tests/golden/stats_{basic,m71}.json hold 20 seeded runs of the REFERENCE
SMCsampler.run() (CPU, float32) on a fixed image (make_golden.py stats):
  basic: 16x16 Poisson ImageModel + ParetoStarPrior(3,3), N=256, K=100, systematic
  m71:   8x8 M71ImageModel + M71Prior(10,10), N=1000, K=100, systematic
  m71_multinomial: the same with multinomial resampling (notebooks/smc.ipynb cell 7)
  m71_mala: 8x8 M71 + M71Prior(4,4), N=500, SingleComponentMALA with K=50, systematic
(make_golden.py passes the M71 flux_detection_threshold to both samplers.)
Random streams cannot match torch's, so parity is distributional: mean log Z
within 1% and within 3 pooled standard errors; non-final ESS = rho*N; final
ESS, posterior mean total flux, pruned-count histogram bins and SMC
iteration counts within 3 pooled standard errors.
"""
import json
import os

import numpy as np
import pytest
import torch

from tests._params import (GOLDEN, M71, p_basic_mh, p_basic_model, p_basic_prior, p_m71_mh,
                           p_m71_model, p_m71_prior)

pytestmark = pytest.mark.gpu
NSEEDS = 60


def _load(which):
    with open(os.path.join(GOLDEN, f"stats_{which}.json")) as f:
        return json.load(f)


# the headline geometry (32x32, S=10, counts_rate 5/40^2) at N=512, K=20, and
# at the headline N=4096 (K=20, and K=100 where the reference runs exist)
# "_oracle": the same configuration run to completion by the CPU restatement
# of the reference's algorithm (tests/golden/make_oracle_stats.py: many more
# seeds than the reference's own 75-minute runs allow; it resolves the log Z
# distribution's lower mode)
C2_MODERATE = ("c2_moderate", "c2_moderate_4096", "c2_moderate_4096_k100",
               "c2_moderate_4096_k100_oracle")
C2_TARGETS = C2_MODERATE + ("c2_reduced",)


def _run(which, cfg, image, seed, fused=True, persist=True):
    from smcdet_amd.sampler import SMCsampler
    torch.manual_seed(seed)
    H, N, S = cfg["tile"], cfg["N"], cfg["S"]
    if which == "basic":
        prior, model, mh = p_basic_prior(H, S, S), p_basic_model(H), p_basic_mh(cfg["K"])
    elif cfg.get("kernel") == "mala":
        from smcdet_amd.kernel import SingleComponentMALA
        prior, model = p_m71_prior(H, S, S), p_m71_model(H)
        mh = SingleComponentMALA(cfg["K"], 0.1, 2.5, M71["flux_lower"], M71["flux_upper"])
    elif which in C2_TARGETS:
        prior, model = p_m71_prior(H, S, S, counts_rate=0.003125), p_m71_model(H)
        mh = p_m71_mh(cfg["K"])
    else:
        prior, model, mh = p_m71_prior(H, S, S), p_m71_model(H), p_m71_mh(cfg["K"])
    # SMCsampler's defaults: incremental MH, persisted rate images refreshed
    # every 8 sweeps, lockstep stopping, speculative fused loop
    s = SMCsampler(image, H, prior, model, mh, N, cfg["rho"], cfg["method"],
                   M71["flux_detection_threshold"], cfg.get("max_smc_iters", 100),
                   print_every=10 ** 9, fused=fused, persist_rate_images=persist)
    esses, taus = [], []
    orig = s._temper_reweight

    def tr(with_resample, orig=orig):
        orig(with_resample)
        esses.append(float(s.ess.flatten()[0]))
        taus.append(float(s.temperature.flatten()[0]))

    s._temper_reweight = tr
    s.run()
    hist = np.bincount(s.pruned_counts.flatten().cpu().numpy(), minlength=S + 1)
    return dict(logZ=float(s.log_normalizing_constant.flatten()[0]), iters=s.iter,
                ess_trace=esses, tau_trace=taus, final_ess=float(s.ess.flatten()[0]),
                pruned_hist=hist / hist.sum(),
                mean_total_flux=float(s.posterior_mean_total_flux(s.fluxes).flatten()[0]),
                # sampler.py:198-219 then :262-266 (make_golden.py's statistic;
                # the weights are uniform after the final resample)
                mean_total_flux_pruned=float(
                    s.posterior_mean_total_flux(s.pruned_fluxes).flatten()[0]),
                # the oracle's statistic (make_oracle_stats.py): the plain mean
                # over the final resampled population
                mean_total_flux_unweighted=float(s.fluxes.sum(-1).mean()))


def _se(a, b):
    return np.sqrt(np.var(a, ddof=1) / len(a) + np.var(b, ddof=1) / len(b))


@pytest.mark.parametrize("which", ["basic", "m71", "m71_multinomial", "m71_mala"])
def test_statistical_parity_vs_reference(which):
    if not os.path.exists(os.path.join(GOLDEN, f"stats_{which}.json")):
        pytest.skip(f"stats_{which}.json not generated")
    ref = _load(which)
    cfg = ref["config"]
    image = torch.tensor(ref["image"], dtype=torch.float32, device="cuda")
    runs = [_run(which, cfg, image, 1000 + i) for i in range(NSEEDS)]
    rr = ref["runs"]
    rho_n = cfg["rho"] * cfg["N"]

    lz, lz_ref = np.array([r["logZ"] for r in runs]), np.array([r["logZ"] for r in rr])
    se = _se(lz, lz_ref)
    diff = lz.mean() - lz_ref.mean()
    assert abs(diff) <= 3 * se, (which, lz.mean(), lz_ref.mean(), se)
    if cfg.get("kernel") != "mala":
        # north_star's 1%: the observed difference may exceed 1% of the
        # reference mean only by sampling noise (2 pooled SE; at m71 the
        # reference's own SE is ~1% of log Z, so the point estimate alone would
        # fail about a third of the time with equal samplers).  SMC with MALA
        # mixes poorly on this image (reference SD ~135 nats): SE test only.
        assert abs(diff) <= 0.01 * abs(lz_ref.mean()) + 2 * se, (which, lz.mean(),
                                                                 lz_ref.mean(), se)

    # every non-final tempering step lands on ESS = rho*N (root of the ESS equation)
    for r in runs:
        inner = np.array(r["ess_trace"][:-1])
        np.testing.assert_allclose(inner, rho_n, rtol=0.01)

    fe, fe_ref = np.array([r["final_ess"] for r in runs]), np.array([r["final_ess"] for r in rr])
    assert abs(fe.mean() - fe_ref.mean()) <= 3 * _se(fe, fe_ref), (fe.mean(), fe_ref.mean())

    it, it_ref = np.array([r["iters"] for r in runs]), np.array([r["iters"] for r in rr])
    assert abs(it.mean() - it_ref.mean()) <= max(3 * _se(it, it_ref), 0.5), (it.mean(),
                                                                             it_ref.mean())

    fl = np.array([r["mean_total_flux"] for r in runs])
    fl_ref = np.array([r["mean_total_flux"] for r in rr])
    assert abs(fl.mean() - fl_ref.mean()) <= 3 * _se(fl, fl_ref), (fl.mean(), fl_ref.mean())

    # pruned-count posterior: per-bin means within 3 pooled SE (the reference's
    # own per-run histograms scatter by up to 0.06 per bin at m71), and total
    # variation <= 0.05 where the reference's runs agree that tightly
    H = np.array([r["pruned_hist"] for r in runs])
    H_ref = np.array([r["pruned_hist"] for r in rr])
    n = max(H.shape[1], H_ref.shape[1])
    H = np.pad(H, ((0, 0), (0, n - H.shape[1])))
    H_ref = np.pad(H_ref, ((0, 0), (0, n - H_ref.shape[1])))
    se_bins = np.sqrt(H.var(0, ddof=1) / len(H) + H_ref.var(0, ddof=1) / len(H_ref))
    d = np.abs(H.mean(0) - H_ref.mean(0))
    assert np.all(d <= 3 * se_bins + 0.01), (H.mean(0).round(3), H_ref.mean(0).round(3))
    if se_bins.max() < 0.01:
        assert 0.5 * d.sum() <= 0.05, (H.mean(0).round(3), H_ref.mean(0).round(3))


@pytest.mark.parametrize("which", C2_TARGETS)
def test_statistical_parity_c2_geometry(which):
    """north_star's "log Z and ESS within 1%" at the headline geometry: one
    32x32 M71 tile, S=10, counts_rate 5/40^2, with the reduced sampler
    (N=512, K=20) of >= 24 reference seeds, and at the
    headline particle count N=4096 (>= 20 reference seeds at K=20; K=100 runs
    when recorded).
      c2_moderate*: four 2-12 nmgy stars; the sampler mixes, log Z has a
        relative spread of ~1% across seeds: mean log Z within 1% and 3 SE,
        ESS = rho*N at every non-final step, final ESS, iteration count and
        total flux within 3 SE.
      c2_reduced: a tile with a 10^4-ADU star, where N=512, K=20 does not mix:
        the reference's own log Z spreads over -5.4e3 .. -3.3e5 (heavy tail),
        so the test is distributional (medians of log Z and iteration counts
        within a bootstrap 99.9% band, two-sample rank test p > 0.001)."""
    from scipy.stats import mannwhitneyu
    if not os.path.exists(os.path.join(GOLDEN, f"stats_{which}.json")):
        pytest.skip(f"stats_{which}.json not generated")
    ref = _load(which)
    cfg = ref["config"]
    image = torch.tensor(ref["image"], dtype=torch.float32, device="cuda")
    n = 48 if cfg["N"] <= 512 else (128 if which.endswith("_oracle") else 40)
    runs = [_run(which, cfg, image, 2000 + i) for i in range(n)]
    rr = ref["runs"]
    rho_n = cfg["rho"] * cfg["N"]
    lz, lz_ref = np.array([r["logZ"] for r in runs]), np.array([r["logZ"] for r in rr])
    it, it_ref = np.array([r["iters"] for r in runs]), np.array([r["iters"] for r in rr])
    # ESS: every non-final step whose increment delta is >= 1e-3 sits on
    # rho*N within 1%, in both samplers.  (Below that, brentq's xtol = 1e-6,
    # which the device Brent iteration reproduces, is not small against delta:
    # the first step's ESS is ~10, not 256 -- compared by mean instead.)
    for r in list(runs) + list(rr):
        e, t = np.array(r["ess_trace"][:-1]), np.array(r["tau_trace"][:-1])
        delta = np.diff(np.concatenate([[0.0], t]))
        np.testing.assert_allclose(e[delta >= 1e-3], rho_n, rtol=0.01)
    e0, e0_ref = np.array([r["ess_trace"][0] for r in runs]), np.array(
        [r["ess_trace"][0] for r in rr])
    assert abs(e0.mean() - e0_ref.mean()) <= 3 * _se(e0, e0_ref), (e0.mean(), e0_ref.mean())
    print(which, "log Z mean", lz.mean(), "ref", lz_ref.mean(), "median", np.median(lz),
          "ref", np.median(lz_ref), "iters", it.mean(), "ref", it_ref.mean())
    if which in C2_MODERATE and len(rr) < 20:
        # a smoke check, not a distributional claim: too few
        # reference runs (8 at K = 100, ~75 min each) to resolve the log Z
        # law's lower mode (~8% of the oracle's 48 runs), so no 3-SE mean
        # gate against them; a rank test and the medians within 1% instead.
        # The distribution-level claim rests on the "_oracle" target (48
        # runs: mean within 3 SE and 1%, rank test, lower-mode share) and on
        # the paired replays of tests/test_gpu_paired.py.
        assert mannwhitneyu(lz, lz_ref).pvalue > 0.001, (np.median(lz), np.median(lz_ref))
        assert abs(np.median(lz) - np.median(lz_ref)) <= 0.01 * abs(np.median(lz_ref))
        assert abs(np.median(it) - np.median(it_ref)) <= max(2.0, 0.15 * np.median(it_ref))
    elif which in C2_MODERATE:
        se = _se(lz, lz_ref)
        diff = lz.mean() - lz_ref.mean()
        assert abs(diff) <= 3 * se, (lz.mean(), lz_ref.mean(), se)
        # pooled SE ~0.3% of log Z here: the 1% criterion is resolved
        assert abs(diff) <= 0.01 * abs(lz_ref.mean()), (lz.mean(), lz_ref.mean())
        fe = np.array([r["final_ess"] for r in runs])
        fe_ref = np.array([r["final_ess"] for r in rr])
        assert abs(fe.mean() - fe_ref.mean()) <= 3 * _se(fe, fe_ref), (fe.mean(), fe_ref.mean())
        assert abs(it.mean() - it_ref.mean()) <= max(3 * _se(it, it_ref), 0.5)
        fkey = "mean_total_flux_unweighted" if which.endswith("_oracle") else "mean_total_flux"
        fl = np.array([r[fkey] for r in runs])
        fl_ref = np.array([r["mean_total_flux"] for r in rr])
        assert abs(fl.mean() - fl_ref.mean()) <= 3 * _se(fl, fl_ref), (fl.mean(), fl_ref.mean())
        if which.endswith("_oracle"):
            # enough seeds on both sides for the distribution's shape: the
            # same law of log Z (rank test) and the same share of runs in the
            # lower mode (two-proportion z test at the midpoint of the modes)
            assert mannwhitneyu(lz, lz_ref).pvalue > 0.001, (np.median(lz), np.median(lz_ref))
            cut = 0.5 * (np.median(lz_ref) + np.percentile(lz_ref, 2))
            p1, p2 = (lz < cut).mean(), (lz_ref < cut).mean()
            pp = (p1 * len(lz) + p2 * len(lz_ref)) / (len(lz) + len(lz_ref))
            se_p = np.sqrt(max(pp * (1 - pp), 1e-12) * (1 / len(lz) + 1 / len(lz_ref)))
            assert abs(p1 - p2) <= 3.3 * se_p, ("lower-mode share", p1, p2, cut)
    else:
        rng = np.random.default_rng(0)
        for a, b in ((lz, lz_ref), (it, it_ref)):
            boot = np.array([np.median(rng.choice(b, b.size)) - np.median(rng.choice(a, a.size))
                             for _ in range(4000)])
            lo, hi = np.quantile(boot, [0.0005, 0.9995])
            assert lo <= 0 <= hi, (np.median(a), np.median(b), lo, hi)
            assert mannwhitneyu(a, b).pvalue > 1e-3


def test_c2_count_posterior():
    """The headline configuration's scientific output (Missing #2):
    the pruned-count posterior (number of detectable in-bounds stars,
    sampler.py:198-219; notebooks/smc.ipynb cell 9 prints the reference's) and
    the pruned posterior mean total flux (sampler.py:262-266), over 256 GPU
    runs of SMCsampler at C2 (32x32 M71 tile, S = 10, N = 4096, K = 100,
    systematic, rho = 0.5) against
      * the 648 float64 oracle runs (stats_c2_moderate_4096_k100_oracle.json),
      * the reference's own 20 runs (stats_c2_moderate_4096_k100.json).
    Gates, pre-registered (tests/_stats.py; fixed before this test ran on a
    GPU): every bin within 3 pooled SE of both targets (the reference side's
    per-run variance floored at the oracle's, tests/_stats.py); total
    variation <= 0.05 against the oracle target; pruned mean
    total flux within 3 pooled SE of both."""
    from tests._stats import count_posterior_compare, hist_var
    orc = _load("c2_moderate_4096_k100_oracle")
    ref = _load("c2_moderate_4096_k100")
    cfg = ref["config"]
    image = torch.tensor(ref["image"], dtype=torch.float32, device="cuda")
    runs = [_run("c2_moderate_4096_k100", cfg, image, 5000 + i) for i in range(256)]
    vs_orc = count_posterior_compare(runs, orc["runs"])
    vs_ref = count_posterior_compare(runs, ref["runs"], var_floor=hist_var(orc["runs"]))
    out = os.environ.get("SMCDET_STATS_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"vs_oracle": vs_orc, "vs_reference": vs_ref}, f, indent=1)
    for name, r in (("oracle", vs_orc), ("reference", vs_ref)):
        print(name, "hist", np.round(r["hist_mean"], 4), "target",
              np.round(r["hist_mean_target"], 4), "z", np.round(r["bin_z"], 2), "TV",
              round(r["total_variation"], 4), "flux", r["pruned_flux"], r["pruned_flux_target"],
              "z", round(r["pruned_flux_z"], 2))
    for name, r in (("oracle", vs_orc), ("reference", vs_ref)):
        assert r["max_abs_bin_z"] <= 3.0, (name, "bin", r["bin_z"])
        assert abs(r["pruned_flux_z"]) <= 3.0, (name, "pruned flux", r["pruned_flux"],
                                                r["pruned_flux_target"])
    assert vs_orc["total_variation"] <= 0.05, ("TV vs oracle", vs_orc["total_variation"])


def test_fused_run_equals_method_by_method_run():
    """run() with the fused schedule (MH gathers the ancestors; one per-tile
    launch does temper + reweight + next resampling indices) consumes the
    random streams in the same order as the method-by-method schedule.  (With
    persisted rate images the fused run starts sweeps from incrementally
    maintained images, which can flip float32 near-tie decisions: that mode is
    checked by test_mh_persisted_rate_images_c2 and the statistical tests.)"""
    ref = _load("basic")
    cfg = ref["config"]
    image = torch.tensor(ref["image"], dtype=torch.float32, device="cuda")
    a = _run("basic", cfg, image, 7, fused=True, persist=False)
    b = _run("basic", cfg, image, 7, fused=False)
    assert a["iters"] == b["iters"]
    assert a["logZ"] == b["logZ"]
    np.testing.assert_array_equal(a["pruned_hist"], b["pruned_hist"])
