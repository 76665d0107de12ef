"""Pins the CPU oracle (oracle/smc_oracle.py) to golden vectors recorded from
the reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import smc_oracle as O
from tests._params import (M71, MALA_FIXTURES, MH_EDGE_FIXTURES, MH_FIXTURES, golden, mala_fixture_setup,
                           mh_fixture_setup, o_basic_model,
                           o_basic_prior, o_m71_mh, o_m71_model, o_m71_prior, tiles_of)


def test_psf_normalizer():
    d = golden("psf.npz")
    assert abs(o_m71_model(8).norm_const - float(d["m71_norm_const_f32"])) <= 2e-6


@pytest.mark.parametrize("H", [8, 16, 32])
def test_psf_dense_m71(H):
    d = golden("psf.npz")
    p = O.psf_dense(d[f"m71_H{H}_locs"], o_m71_model(H))
    np.testing.assert_allclose(p, d[f"m71_H{H}_psf"], rtol=1e-6, atol=2e-8)


def test_psf_dense_basic():
    d = golden("psf.npz")
    p = O.psf_dense(d["m71_H16_locs"], o_basic_model(16))
    np.testing.assert_allclose(p, d["basic_H16_psf"], rtol=1e-6, atol=1e-7)


def test_psf_profiles():
    d = golden("psf.npz")
    r2 = d["m71_r"].astype(np.float64) ** 2
    m = o_m71_model(8)
    np.testing.assert_allclose(O.m71_psf_unnormalized(r2, m.psf_params), d["m71_unnorm"],
                               rtol=2e-6, atol=1e-12)
    np.testing.assert_allclose(m.psf_value(r2), d["m71_norm"], rtol=2e-6, atol=1e-12)
    np.testing.assert_allclose(o_basic_model(8).psf_value(r2), d["basic_norm"], rtol=2e-6,
                               atol=1e-12)


@pytest.mark.parametrize("key,H", [("m71_H8_S10", 8), ("m71_H32_S10", 32), ("m71_H16_S3", 16)])
def test_loglik_m71(key, H):
    d = golden("loglik.npz")
    ll = O.loglikelihood(d[key + "_image"][None, None], d[key + "_locs"], d[key + "_fluxes"],
                         o_m71_model(H))
    # reference float32 vs float64 oracle: relative rounding of a 1,024-term sum
    np.testing.assert_allclose(ll, d[key + "_loglik"], rtol=1e-6, atol=2e-2)
    np.testing.assert_allclose(ll, d[key + "_loglik_f64"], rtol=1e-7, atol=1e-3)
    lp = O.log_prior(d[key + "_counts"], d[key + "_locs"], d[key + "_fluxes"],
                     o_m71_prior(H, int(d[key + "_counts"].max()), int(d[key + "_counts"].max())))
    np.testing.assert_allclose(lp, d[key + "_logprior"], rtol=1e-6, atol=1e-4)


def test_loglik_m71_tiles():
    d = golden("loglik.npz")
    ll = O.loglikelihood(tiles_of(d["m71_tiles_image"], 8), d["m71_tiles_locs"],
                         d["m71_tiles_fluxes"], o_m71_model(8))
    np.testing.assert_allclose(ll, d["m71_tiles_loglik"], rtol=1e-6, atol=2e-2)


@pytest.mark.parametrize("key", ["basic_H16_S3", "basic_bright"])
def test_loglik_poisson(key):
    d = golden("loglik.npz")
    ll = O.loglikelihood(d[key + "_image"][None, None], d[key + "_locs"], d[key + "_fluxes"],
                         o_basic_model(16))
    np.testing.assert_allclose(ll, d[key + "_loglik"], rtol=1e-6, atol=2e-2)


def test_log_prior():
    d = golden("prior.npz")
    lp = O.log_prior(d["m71_counts"], d["m71_locs"], d["m71_fluxes"],
                     o_m71_prior(8, 0, 12, counts_rate=0.01))
    np.testing.assert_allclose(lp, d["m71_logprior"], rtol=1e-6, atol=1e-4)
    lp = O.log_prior(d["basic_counts"], d["basic_locs"], d["basic_fluxes"],
                     o_basic_prior(16, 3, 3))
    np.testing.assert_allclose(lp, d["basic_logprior"], rtol=1e-6, atol=1e-4)


def test_prior_sample_stratified():
    d = golden("prior.npz")
    pr = o_m71_prior(8, 3, 5)
    c, l, f = O.prior_sample_stratified(pr, 2, 8, d["m71_strat_uloc"], d["m71_strat_uflux"])
    np.testing.assert_array_equal(c, d["m71_strat_counts"])
    np.testing.assert_allclose(l, d["m71_strat_locs"], rtol=0, atol=4e-6)
    np.testing.assert_allclose(f, d["m71_strat_fluxes"], rtol=4e-6, atol=0)
    lp = O.log_prior(c, l, f, pr)
    np.testing.assert_allclose(lp, d["m71_strat_logprior"], rtol=1e-6, atol=1e-4)


def test_truncated_normal():
    d = golden("distributions.npz")
    sl = float(np.float32(0.1))
    x = O.tn_sample(d["loc_mu"].astype(np.float64), sl, -4.0, 36.0, d["loc_u"])
    np.testing.assert_allclose(x, d["loc_x"], rtol=1e-7, atol=1e-5 * sl + 4e-6)
    np.testing.assert_allclose(
        O.tn_log_prob(d["loc_x"].astype(np.float64), d["loc_mu"].astype(np.float64), sl, -4.0,
                      36.0), d["loc_logprob_x"], rtol=1e-6, atol=1e-5)
    lb, ub = float(np.float32(M71["flux_lower"])), float(np.float32(M71["flux_upper"]))
    x = O.tn_sample(d["flux_mu"].astype(np.float64), 2.5, lb, ub, d["flux_u"])
    np.testing.assert_allclose(x, d["flux_x"], rtol=1e-7, atol=2e-5 * 2.5)
    np.testing.assert_allclose(
        O.tn_log_prob(d["flux_x"].astype(np.float64), d["flux_mu"].astype(np.float64), 2.5, lb,
                      ub), d["flux_logprob_x"], rtol=1e-6, atol=1e-5)


def test_truncated_pareto():
    d = golden("distributions.npz")
    a, L, U = M71["flux_alpha"], M71["flux_lower"], M71["flux_upper"]
    np.testing.assert_allclose(O.trunc_pareto_sample(d["tpareto_u"], a, L, U), d["tpareto_x"],
                               rtol=1e-5)
    np.testing.assert_allclose(O.trunc_pareto_log_prob(d["tpareto_x"].astype(np.float64), a, L, U),
                               d["tpareto_logprob"], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("name", MH_FIXTURES)
def test_mh_sweep_replay(name):
    d = golden(name + ".npz")
    td, model, prior, mh = mh_fixture_setup(name)
    t = tiles_of(d["image"], td)
    tau = np.full(t.shape[:2], float(d["tau"]))
    lt0 = O.log_target(t, d["counts"], d["locs0"], d["fluxes0"], tau, prior, model)
    np.testing.assert_allclose(lt0, d["init_logtarget"], rtol=1e-6, atol=2e-2)
    l, f, acc = O.mh_sweep(t, d["counts"], d["locs0"], d["fluxes0"], tau, prior, model, mh,
                           d["comp"], d["uloc"], d["uflux"], d["uacc"])
    np.testing.assert_allclose(l, d["locs1"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(f, d["fluxes1"], rtol=1e-6, atol=5e-4)
    np.testing.assert_array_equal(acc.astype(np.float32), d["acc"])


def test_temper_update_weights():
    d = golden("smc_steps.npz")
    for dt in (np.float64, np.float32):
        tau, delta = O.temper(d["temper_loglik"], d["temper_tau_in"], float(d["temper_rho_N"]), dt)
        np.testing.assert_allclose(tau, d["temper_tau_out"], rtol=0, atol=2e-6)
        np.testing.assert_allclose(delta, d["temper_delta"], rtol=0, atol=2e-6)
    W, ess, lz = O.update_weights(d["temper_loglik"], d["temper_tau_out"], d["temper_tau_in"],
                                  d["weights_logZ_in"], 512)
    np.testing.assert_allclose(W, d["weights_W"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(ess, d["weights_ess"], rtol=1e-5)
    np.testing.assert_allclose(lz, d["weights_logZ"], rtol=1e-6, atol=1e-4)


def test_systematic_resample_exact():
    d = golden("smc_steps.npz")
    np.testing.assert_array_equal(O.systematic_resample_index(d["resample_W"], d["resample_U"]),
                                  d["resample_idx"])
    np.testing.assert_array_equal(
        O.systematic_resample_index(d["resample_hand_W"], d["resample_hand_U"]),
        d["resample_hand_idx"])


def test_prune_exact():
    d = golden("smc_steps.npz")
    pc, pl, pf = O.prune(d["prune_locs"], d["prune_fluxes"], int(d["prune_tile_dim"]),
                         float(d["prune_threshold"]))
    np.testing.assert_array_equal(pc, d["prune_counts"])
    np.testing.assert_array_equal(pl, d["prune_out_locs"])
    np.testing.assert_array_equal(pf, d["prune_out_fluxes"])


@pytest.mark.parametrize("name", ["smc_replay_m71_8x8", "smc_replay_m71_tiles"])
def test_smc_end_to_end_replay(name):
    d = golden(name + ".npz")
    S, K, N = int(d["S"]), int(d["K"]), int(d["N"])
    r = O.smc_run_replay(d["image"], int(d["tile_dim"]), o_m71_prior(8, S, S), o_m71_model(8),
                         o_m71_mh(K), N, O.DrawStream(d),
                         flux_detection_threshold=M71["flux_detection_threshold"])
    assert r["iters"] == int(d["iters"])
    np.testing.assert_allclose(r["logZ"], d["logZ"], rtol=1e-5)
    np.testing.assert_allclose(r["ess"], d["ess"], rtol=1e-4)
    np.testing.assert_allclose(r["trace"]["tau"], d["trace_tau"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(r["locs"], d["locs"], rtol=0, atol=2e-5)
    np.testing.assert_array_equal(r["pruned_counts"], d["pruned_counts"])


@pytest.mark.parametrize("name", MH_FIXTURES)
def test_c_oracle_mh_replay(name):
    """The C restatement (bench.py's CPU baseline) replays the reference's
    recorded MH draws to the same states and accept decisions."""
    from oracle import c_oracle
    d = golden(name + ".npz")
    td, model, prior, mh = mh_fixture_setup(name)
    t = tiles_of(d["image"], td)
    replay = {k: d[k] for k in ("comp", "uloc", "uflux", "uacc")}
    l, f, acc = c_oracle.mh_sweep(t, d["counts"], d["locs0"], d["fluxes0"], float(d["tau"]),
                                  prior, model, mh, replay=replay, threads=2)
    np.testing.assert_allclose(l, d["locs1"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(f, d["fluxes1"], rtol=1e-6, atol=5e-4)
    np.testing.assert_array_equal(acc.astype(np.float32), d["acc"])


@pytest.mark.parametrize("name", MALA_FIXTURES)
def test_c_oracle_mala_replay(name):
    """The C MALA restatement (smcdet/kernel.py:133-275) replays the
    reference's recorded draws: the same gradients as torch.autograd.grad, the
    same proposals, accept decisions and final states.  The tau=1 and tile
    fixtures include proposal means far outside the box (float32 mass-in-box
    underflow) and proposals clamped to the box edge."""
    from oracle import c_oracle
    d = golden(name + ".npz")
    td, model, prior, mala = mala_fixture_setup(name)
    t = tiles_of(d["image"], td)
    replay = {k: d[k] for k in ("comp", "uloc", "uflux", "uacc")}
    l, f, acc, g, prop = c_oracle.mala_sweep(t, d["counts"], d["locs0"], d["fluxes0"],
                                             float(d["tau"]), prior, model, mala, replay=replay,
                                             threads=2, record=True)
    gc = d["grad_cur"]
    scale = np.abs(gc).max(axis=tuple(range(gc.ndim - 1)))
    # iteration 0 (identical states): the analytic gradient vs autograd, to the
    # reference's float32 summation error (~1e-7 x the summed |terms|)
    np.testing.assert_array_less(np.abs(g[0] - gc[0]), 1e-4 * np.abs(gc[0]) + 1e-4 * scale + 1e-6)
    # later iterations: states agree to float32 rounding, which the MALA drift
    # (step^2/2 x gradient) can amplify to ~1e-3 relative before a proposal
    np.testing.assert_array_less(np.abs(g - gc), 2e-2 * np.abs(gc) + 1e-4 * scale + 1e-6)
    np.testing.assert_allclose(prop, d["proposal"], rtol=1e-6, atol=1e-3)
    np.testing.assert_allclose(l, d["locs1"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(f, d["fluxes1"], rtol=1e-6, atol=1e-3)
    np.testing.assert_array_equal(acc.astype(np.float32), d["acc"])


@pytest.mark.parametrize("name,td,S", [("mcmc_m71_8x8", 8, 4), ("mcmc_m71_tiles", 8, 3)])
def test_c_oracle_mh_chain_replay(name, td, S):
    """MHsampler (smcdet/sampler.py:301-493) = one single-component MH chain
    per tile at temperature 1: the C restatement replays the reference's
    recorded draws to the same kept samples and accept flags."""
    from oracle import c_oracle
    d = golden(name + ".npz")
    t = tiles_of(d["image"], td)
    nt = t.shape[0]
    replay = {k: d[k] for k in ("comp", "uloc", "uflux", "uacc")}
    l, f, acc = c_oracle.mh_chain(t, np.full((nt, nt), S, np.float32), d["init_locs"],
                                  d["init_fluxes"], o_m71_prior(td, S, S), o_m71_model(td),
                                  o_m71_mh(1), int(d["total"]), int(d["burnin"]), int(d["keep"]),
                                  replay)
    np.testing.assert_array_equal(acc, d["accept"])
    np.testing.assert_allclose(l, d["locs"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(f, d["fluxes"], rtol=1e-6, atol=1e-4)


@pytest.mark.parametrize("name", MH_EDGE_FIXTURES)
def test_mh_edge_decisions_replay(name):
    """Every accept decision of the reference's upper-edge fixture
    (make_golden.py gen_mh_edge): the proposal that lands on the prior box's
    upper edge is rejected and every later proposal of that particle too (the
    NaN cache of kernel.py:125); the control particles keep moving."""
    d = golden(name + ".npz")
    td, model, prior, mh = mh_fixture_setup(name)
    t = tiles_of(d["image"], td)
    tau = np.full(t.shape[:2], float(d["tau"]))
    _, _, _, _, acc_tr = O.mh_sweep(t, d["counts"], d["locs0"], d["fluxes0"], tau, prior, model,
                                    mh, d["comp"], d["uloc"], d["uflux"], d["uacc"], trace=True)
    np.testing.assert_array_equal(acc_tr, d["accept"])
    hit = d["edge_hit"]
    first = np.where(hit.any(0), hit.argmax(0), hit.shape[0])
    frozen = np.arange(hit.shape[0])[:, None, None, None] >= first[None]
    assert frozen.sum() > 0 and not d["accept"][frozen].any()
    # without the freeze the edge proposal is still rejected, but the particle
    # moves on: the final states of the frozen particles differ
    l2, _, _, _, acc2 = O.mh_sweep(t, d["counts"], d["locs0"], d["fluxes0"], tau, prior, model,
                                   mh, d["comp"], d["uloc"], d["uflux"], d["uacc"], trace=True,
                                   edge_freeze=False)
    assert not acc2[hit].any()
    assert acc2[frozen].any()


def test_c_oracle_mh_chain_edge_freeze():
    """The C restatement replays the reference's frozen MHsampler chains
    (make_golden.py gen_mcmc_edge): every accept flag and kept sample."""
    from oracle import c_oracle
    d = golden("mcmc_m71_edge_tiles.npz")
    img = tiles_of(d["image"], 8)
    replay = {k: d[k] for k in ("comp", "uloc", "uflux", "uacc")}
    l, f, acc = c_oracle.mh_chain(img, np.full((2, 2), 3, np.float32), d["init_locs"],
                                  d["init_fluxes"], o_m71_prior(8, 3, 3), o_m71_model(8),
                                  o_m71_mh(1), int(d["total"]), int(d["burnin"]), int(d["keep"]),
                                  replay)
    np.testing.assert_array_equal(acc, d["accept"])
    np.testing.assert_allclose(l, d["locs"], rtol=0, atol=1e-5)
    plan = d["edge_plan"]
    for th, tw, j, k in plan:
        assert d["accept"][th, tw, k:].sum() == 0


def _steps4096_cases():
    d = golden("smc_steps_4096.npz")
    return d, [{k[4:]: d[k] for k in d.files if k.startswith(f"c{i:02d}_")}
               for i in range(int(d["n_cases"]))]


def test_tile_pass_4096_oracle():
    """The reference's temper / update_weights / systematic resampling at the
    headline N=4096 (make_golden.py gen_smc_steps_4096: the log-likelihoods
    of a real 32x32 S=10 run, temperature 0 -> 0.14, plus temperatures near 1
    and a root 1e-5 above tau=0.99): the oracle's Brent reproduces brentq's
    increments, its weights / ESS / log Z and its indices the reference's."""
    d, cases = _steps4096_cases()
    assert len(cases) >= 12
    for c in cases:
        ll = c["loglik"].reshape(1, 1, -1)
        tau_in = c["tau_in"].reshape(1, 1)
        tau, _ = O.temper(ll, tau_in, float(d["rho_N"]))
        np.testing.assert_allclose(tau.ravel(), c["tau_out"].ravel(), rtol=0, atol=2e-6)
        W, ess, lz = O.update_weights(ll, c["tau_out"].reshape(1, 1), tau_in,
                                      c["logZ_in"].reshape(1, 1), ll.shape[-1])
        np.testing.assert_allclose(W.ravel(), c["W"], rtol=1e-5, atol=1e-12)
        np.testing.assert_allclose(float(ess.ravel()[0]), float(c["ess"]), rtol=1e-5)
        np.testing.assert_allclose(float(lz.ravel()[0]), float(c["logZ"]), rtol=1e-6, atol=1e-4)
        if "idx" in c:
            idx = O.systematic_resample_index(c["W"].reshape(1, 1, -1), c["U"].reshape(1, 1))
            np.testing.assert_array_equal(idx.ravel(), c["idx"])


def test_c_oracle_teacher_forced_c2():
    """The C restatement replays the reference's recorded headline-geometry
    sweeps (make_golden.py gen_mh_teacher: 32x32, S=10, N=1024, K=100, three
    SMC iterations): every particle whose decisions the float64 oracle makes
    with margins >= 1e-4 ends in the reference's state."""
    from oracle import c_oracle
    d = golden("mh_teacher_c2.npz")
    K = int(d["K"])
    prior, model = o_m71_prior(32, 10, 10, counts_rate=0.003125), o_m71_model(32)
    mh = o_m71_mh(K)
    img = d["image"].reshape(1, 1, 32, 32)
    for i in range(len(d["steps"])):
        k = f"s{i}_"
        replay = {"comp": d[k + "comp"].astype(np.int32), "uloc": d[k + "uloc"],
                  "uflux": d[k + "uflux"], "uacc": d[k + "uacc"]}
        l1, f1, _ = c_oracle.mh_sweep(img, d[k + "counts"], d[k + "locs0"], d[k + "fluxes0"],
                                      float(d[k + "tau"]), prior, model, mh, replay=replay)
        full = d[k + "pin"] == K
        assert full.mean() > 0.98
        np.testing.assert_allclose(l1[0, 0][full], d[k + "locs1"][0, 0][full], rtol=0, atol=2e-5)
        np.testing.assert_allclose(f1[0, 0][full], d[k + "fluxes1"][0, 0][full], rtol=2e-6,
                                   atol=1e-3)
