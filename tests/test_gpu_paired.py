"""Paired (same-draws) whole runs at the headline configuration (VERDICT r3
"next" #2): one 32x32 M71 tile, S=10, N=4096, K=100, rho=0.5, systematic.

tests/golden/stats_c2_moderate_4096_k100_oracle.json holds 48 complete runs
of the CPU restatement (tests/golden/make_oracle_stats.py: the float64 C sweep
with full re-renders, brentq tempering, softmax, systematic resampling) with
their own seeded streams: numpy PCG64 for the prior draw and the systematic
offsets, splitmix64 per particle and SMC iteration in the sweep.  Here the
GPU sampler replays exactly those draws (oracle.c_oracle.sweep_draws, pinned
against the C sweep by tests/test_oracle_paired.py) through the reference's
loop (smcdet/sampler.py:221-256: resample -> mutate -> temper ->
update_weights), so each GPU run is the oracle run's twin.

Twins part where a float32 decision differs from the float64 one (a near
tie among ~7M decisions per run): the temperature ladders agree for the
first iterations and leave each other at iteration 3-12
(scripts/paired_bisect.py, profiles/r04/paired_bisect.json) -- in every
variant, the reference's own float32 full re-render and a GPU run tempered
by the oracle's float64 tile pass included.  From there on a twin is a new
draw of the run's random outcome, so on "fragile" seeds (oracle log Z
between the modes) the mode is not a function of the draws.

The null rate of mode discordance is ORACLE-ONLY evidence, frozen in round 6
(pre-registered; never re-fitted to GPU replays): on the 276 seeds that both
committed oracle targets hold, the float64 oracle and its float32-class build
(same draws, stats_c2_moderate_4096_k100_oracle{,_f32}.json) end in different
modes in 19 runs (10 : 9) -- the chaos of near-tie decisions between two
arithmetics of the same algorithm, with no implementation under test in it
(tests/test_oracle_paired.py::test_oracle_only_discordance_rate recomputes it
from the fixtures).  The GPU-vs-oracle replays of rounds 4-5 (14 of 257, 30 of
648) are supporting evidence only.  The test checks:
  * the pairing: ladders equal (|delta tau| <= 1e-5) for the first two
    iterations in >= 90% of runs;
  * agreement where runs are robust: the number of pairs in different modes
    (cut: median - 40 nats; the lower mode sits ~65-80 nats below) is
    consistent with that oracle-only rate (one-sided binomial p > 0.001),
    and median |delta log Z| <= 5 nats over the runs in the same mode;
  * no systematic excess: McNemar's exact test on the runs in different
    modes (GPU lower only vs oracle lower only), two-sided p > 0.01.
The reference-arithmetic twin (SingleComponentMH(full_recompute=True)) is
recorded next to it as a control (SMCDET_PAIRED_OUT summary).
"""
# FROZEN (round 6): the oracle-only discordance, float64 vs float32-class
# oracle on their 276 common seeds.  Do not re-fit.
DISCORDANCE = 19 / 276
import json
import os

import numpy as np
import pytest
import torch

from tests._params import GOLDEN, M71, p_m71_mh, p_m71_model, p_m71_prior

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TARGET = "stats_c2_moderate_4096_k100_oracle.json"
# (SMCDET_PAIRED_CHUNKS: more, shorter tests when every oracle run is replayed)
CHUNKS = int(os.environ.get("SMCDET_PAIRED_CHUNKS", "4"))
_results = {}


def _target():
    """The oracle runs replayed: the first 48 seeds by default (the round-end
    suite's budget); SMCDET_PAIRED_ALL=1 replays every run of the target
    (hundreds since round 5: make_oracle_stats.py on the GPU boxes' host
    cores)."""
    with open(os.path.join(GOLDEN, TARGET)) as f:
        doc = json.load(f)
    if os.environ.get("SMCDET_PAIRED_ALL") != "1":
        doc["runs"] = sorted(doc["runs"], key=lambda r: r["seed"])[:48]
    elif os.environ.get("SMCDET_PAIRED_PART"):
        # "k/P": the k-th of P interleaved parts of every run (one GPU call
        # each; scripts/paired_combine.py pools the parts' per-run results)
        k, P = (int(x) for x in os.environ["SMCDET_PAIRED_PART"].split("/"))
        doc["runs"] = sorted(doc["runs"], key=lambda r: r["seed"])[k::P]
    return doc


def paired_gpu_run(img, cfg, seed, full_recompute=False):
    """make_oracle_stats.run_one's schedule and streams on the GPU sampler."""
    from oracle import c_oracle as C
    from smcdet_amd.sampler import SMCsampler
    H, N, S, K = cfg["tile"], cfg["N"], cfg["S"], cfg["K"]
    prior = p_m71_prior(H, S, S, counts_rate=cfg["counts_rate"])
    model, mh = p_m71_model(H), p_m71_mh(K, full_recompute=full_recompute)
    image = torch.tensor(img, dtype=torch.float32, device=DEV)
    s = SMCsampler(image, H, prior, model, mh, N, cfg["rho"], "systematic",
                   M71["flux_detection_threshold"], cfg["max_smc_iters"], print_every=10 ** 9,
                   device=DEV)
    rng = np.random.default_rng(seed)
    uloc = torch.from_numpy(rng.random((1, 1, N, S, 2), dtype=np.float32)).to(DEV)
    uflux = torch.from_numpy(rng.random((1, 1, N, S), dtype=np.float32)).to(DEV)
    s.counts, s.locs, s.fluxes = prior.sample_stratified(1, N, device=DEV, uloc=uloc, uflux=uflux)
    s.temperature_prev = torch.zeros(1, 1, device=DEV)
    s.temperature = torch.zeros(1, 1, device=DEV)
    s.log_normalizing_constant = torch.zeros(1, 1, device=DEV)
    s._fresh_loglik = None
    s.temper()
    s.update_weights()
    s.iter = 0
    taus = [float(s.temperature.flatten()[0])]
    while bool((s.temperature < 1).any()) and s.iter <= s.max_smc_iters:
        s.iter += 1
        u = torch.from_numpy(rng.random((1, 1), dtype=np.float32)).to(DEV)
        idx = s.resample_index(u=u)
        d = C.sweep_draws((seed * 1000003 + s.iter) & 0xFFFFFFFFFFFF, 1, N, K, S)
        replay = {k: torch.from_numpy(v.reshape((K, 1, 1) + v.shape[2:])) for k, v in d.items()}
        s.locs, s.fluxes, s.mutation_acc_rates = mh.run(
            s.tiled_image, s.counts, s.locs, s.fluxes, s.temperature, s.log_target,
            ancestors=idx, replay=replay)
        s.counts = mh.last_counts
        s._fresh_loglik = mh.last_loglik
        s.temper()
        s.update_weights()
        taus.append(float(s.temperature.flatten()[0]))
    return dict(seed=seed, logZ=float(s.log_normalizing_constant.flatten()[0]), iters=s.iter,
                final_ess=float(s.ess.flatten()[0]), tau=taus)


@pytest.mark.parametrize("chunk", range(CHUNKS))
def test_paired_runs_chunk(chunk):
    ref = _target()
    runs = ref["runs"]
    # SMCDET_PAIRED_NO_TWIN=1 (the every-run replays): no full-recompute control
    twin = os.environ.get("SMCDET_PAIRED_NO_TWIN") != "1"
    for r in runs[chunk::CHUNKS]:
        out = paired_gpu_run(ref["image"], ref["config"], r["seed"])
        full = (paired_gpu_run(ref["image"], ref["config"], r["seed"], full_recompute=True)
                if twin else {"logZ": float("nan"), "iters": -1})
        out["full_logZ"], out["full_iters"] = full["logZ"], full["iters"]
        out["oracle_logZ"], out["oracle_iters"] = r["logZ"], r["iters"]
        ot, gt = r["tau_trace"], out["tau"]
        n = min(len(ot), len(gt))
        off = [i for i in range(n) if abs(ot[i] - gt[i]) > 1e-5]
        out["first_tau_divergence"] = off[0] if off else n
        _results[r["seed"]] = out
        print(f"seed {r['seed']}: GPU log Z {out['logZ']:.2f} ({out['iters']} it), full re-render "
              f"{full['logZ']:.2f}, oracle {r['logZ']:.2f} ({r['iters']} it); ladders part at "
              f"iteration {out['first_tau_divergence']}", flush=True)


def _mcnemar_p(b, c):
    """Exact two-sided McNemar p-value for b vs c discordant pairs."""
    from math import comb
    n, k = b + c, min(b, c)
    if n == 0:
        return 1.0
    return min(1.0, 2.0 * sum(comb(n, i) for i in range(k + 1)) / 2.0 ** n)


def _compare(lz, lz_o, cut):
    low, low_o = lz < cut, lz_o < cut
    same = low == low_o
    d = lz - lz_o
    b, c = int((low & ~low_o).sum()), int((~low & low_o).sum())
    return dict(same_mode=int(same.sum()), lower_only_here=b, lower_only_oracle=c,
                mcnemar_p=_mcnemar_p(b, c), lower_mode=int(low.sum()),
                lower_mode_oracle=int(low_o.sum()),
                abs_dlogz_median_same_mode=float(np.median(np.abs(d[same]))),
                abs_dlogz_p90=float(np.percentile(np.abs(d), 90)), mean_dlogz=float(d.mean()))


def test_paired_runs_same_mode():
    ref = _target()
    runs = ref["runs"]
    if len(_results) < len(runs):
        pytest.skip("needs every chunk of test_paired_runs_chunk")
    lz_o = np.array([r["logZ"] for r in runs])
    cut = float(np.median(lz_o) - 40.0)
    res = [_results[r["seed"]] for r in runs]
    gpu = _compare(np.array([x["logZ"] for x in res]), lz_o, cut)
    has_twin = all(np.isfinite(x["full_logZ"]) for x in res)
    full = _compare(np.array([x["full_logZ"] for x in res]), lz_o, cut) if has_twin else None
    twins = _compare(np.array([x["logZ"] for x in res]), np.array([x["full_logZ"] for x in res]),
                     cut) if has_twin else None
    first = np.array([x["first_tau_divergence"] for x in res])
    summary = dict(cut=cut, n=len(res), gpu_vs_oracle=gpu, full_recompute_vs_oracle=full,
                   gpu_vs_full_recompute=twins,
                   ladder_first_divergence={"min": int(first.min()),
                                            "median": float(np.median(first)),
                                            "share_ge_2": float((first >= 2).mean())},
                   runs=res)
    path = os.environ.get("SMCDET_PAIRED_OUT")
    if path:
        with open(path, "w") as f:
            json.dump(summary, f, indent=1)
    print({k: v for k, v in summary.items() if k != "runs"})
    from scipy.stats import binomtest
    assert (first >= 2).mean() >= 0.9, summary["ladder_first_divergence"]
    discordant = len(res) - gpu["same_mode"]
    assert binomtest(discordant, len(res), DISCORDANCE, alternative="greater").pvalue > 0.001, gpu
    assert gpu["abs_dlogz_median_same_mode"] <= 5.0, gpu
    assert gpu["mcnemar_p"] > 0.01, gpu
